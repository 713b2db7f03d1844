// lgs_launch.h -- host-side launch interface between the runtime
// (lgs_api.cpp) and the kernels (lgs_encode.hip, lgs_decode.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lgs {

struct DecodeArgs {
  const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
  uint8_t* out; const uint64_t* out_off; const uint32_t* out_cap;
  uint32_t* out_len; uint8_t* status; const uint32_t* index; uint32_t n;
};

struct EncodeArgs {
  const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
  uint8_t* out; const uint64_t* out_off; uint32_t* out_len;
  const uint32_t* hdr; const uint32_t* index; uint32_t n;
};

// max_out: largest out_cap in the launch (selects the LDS class).
hipError_t launch_decode(const DecodeArgs& a, uint32_t max_out, hipStream_t s);
// max_in: largest item length in the launch (<= 65536).
hipError_t launch_encode(const EncodeArgs& a, uint32_t max_in, hipStream_t s);
// Several-blocks-per-wave encoder (lgs_encode_group.hip); lanes per block =
// 16, 32 or 64.  hipErrorNotSupported if the batch does not qualify.
hipError_t launch_encode_group(const EncodeArgs& a, uint32_t max_in, uint32_t lanes,
                               hipStream_t s);
hipError_t launch_concat(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                         uint8_t* dst, const uint64_t* dst_off, uint32_t n, hipStream_t s);

}  // namespace lgs
