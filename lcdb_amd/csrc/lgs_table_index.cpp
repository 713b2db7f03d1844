// lgs_table_index.cpp -- opening a table file for the batched read path
// (SURVEY.md §8(f) row 3): the footer, the index block's data-block handles
// and the metaindex's filter handle, as lcdb's table code reaches them
// (src/table/table.c:78-180, format.c:116-150, block.c:49-130, 255-297,
// 412-450).  Host code: the footer and the entry walk are a few hundred
// bytes of varints per table; the index and metaindex blocks themselves are
// read (checksum, type, Snappy) by the device path, lgs_table_read_host.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/lcdb_gpu_snappy.h"

#include "lgs_launch.h"

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;   // format.h:39
constexpr size_t kFooterSize = 48;                        // format.h:31

uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

// coding.h:170-204.
bool varint32(uint32_t* z, const uint8_t** p, size_t* n) {
  uint32_t r = 0;
  for (uint32_t sh = 0; sh <= 28 && *n > 0; sh += 7) {
    const uint32_t b = **p;
    ++*p;
    --*n;
    if (b & 128) {
      r |= (b & 127) << sh;
    } else {
      r |= b << sh;
      *z = r;
      return true;
    }
  }
  return false;
}

// coding.h:238-260.
bool varint64(uint64_t* z, const uint8_t** p, size_t* n) {
  uint64_t r = 0;
  for (uint32_t sh = 0; sh <= 63 && *n > 0; sh += 7) {
    const uint64_t b = **p;
    ++*p;
    --*n;
    if (b & 128) {
      r |= (b & 127) << sh;
    } else {
      r |= b << sh;
      *z = r;
      return true;
    }
  }
  return false;
}

// format.c:66-80 (trailing bytes ignored).
bool handle_import(uint64_t* off, uint64_t* size, const uint8_t* p, size_t n) {
  return varint64(off, &p, &n) && varint64(size, &p, &n);
}

// One block through the device read path: contents, or the read status.
int read_block(const uint8_t* file, uint64_t file_len, uint64_t off, uint64_t size, int verify,
               std::vector<uint8_t>* out, uint8_t* st) {
  // Output capacity: the raw size, or the Snappy size header (snappy.c:386-399)
  // when the type byte says Snappy; a bad header fails in the read itself.
  uint32_t cap = 0;
  if (size <= 0xffffffffull) cap = (uint32_t)size;
  if (off < file_len && size < file_len - off && file[off + size] == LGS_SNAPPY_COMPRESSION) {
    const uint8_t* p = file + off;
    size_t n = (size_t)size;
    uint32_t want = 0;
    cap = varint32(&want, &p, &n) ? want : 0;
  }
  out->assign((size_t)cap + 16, 0);
  const uint64_t out_off = 0;
  uint32_t out_len = 0;
  const int rc = lgs_table_read_host(file, file_len, &off, &size, 1, verify, out->data(),
                                     &out_off, &cap, &out_len, st);
  if (rc != LGS_OK) return rc;
  out->resize(*st == LGS_ST_OK ? out_len : 0);
  return LGS_OK;
}

// block.c:49-70 + ldb_blockiter_create (:428-451) + first/next (:255-297,
// 412-415): visit(key, value) per entry from restart point 0 on.  Returns
// LGS_ST_OK at the end of the block, LGS_ST_CORRUPT at a bad block or entry
// ("bad block contents" / "bad entry in block").
template <class Visit>
uint8_t walk_block(const std::vector<uint8_t>& b, bool internal_keys, Visit visit) {
  const size_t size = b.size();
  if (size < 4) return LGS_ST_CORRUPT;
  const uint32_t nr = le32(b.data() + size - 4);
  if (nr > (size - 4) / 4) return LGS_ST_CORRUPT;          // block.c:62-65
  if (nr == 0) return LGS_ST_OK;                          // empty iterator (:439-440)
  const uint32_t restarts = (uint32_t)(size - (1 + (size_t)nr) * 4);
  uint32_t cur = le32(b.data() + restarts);               // get_restart_point(0) (:157-166)
  if (cur > restarts) cur = restarts;
  std::string key;
  const uint8_t* const data = b.data();
  for (;;) {
    if (cur >= restarts) return LGS_ST_OK;
    const uint8_t* p = data + cur;
    size_t n = restarts - cur;
    if (n < 3) return LGS_ST_CORRUPT;                     // decode_entry (:80-126)
    uint32_t shared = p[0], non_shared = p[1], vlen = p[2];
    if ((shared | non_shared | vlen) < 128) {
      p += 3;
      n -= 3;
    } else if (!varint32(&shared, &p, &n) || !varint32(&non_shared, &p, &n) ||
               !varint32(&vlen, &p, &n)) {
      return LGS_ST_CORRUPT;
    }
    if (n < (uint64_t)non_shared + vlen) return LGS_ST_CORRUPT;
    if (key.size() < shared) return LGS_ST_CORRUPT;       // parse_next_key (:266-273)
    if (internal_keys && (uint64_t)shared + non_shared < 8) return LGS_ST_CORRUPT;
    key.resize(shared);
    key.append((const char*)p, non_shared);
    visit(key, p + non_shared, (size_t)vlen);
    cur = (uint32_t)(p + non_shared + vlen - data);
  }
}

}  // namespace

extern "C" int lgs_table_index_host(const uint8_t* file, uint64_t file_len, int paranoid_checks,
                                    int internal_keys, const char* filter_name,
                                    uint64_t* handle_off, uint64_t* handle_size, uint32_t cap,
                                    uint32_t* count, uint8_t* keys, size_t keys_cap,
                                    uint64_t* key_off, uint64_t* filter_off,
                                    uint64_t* filter_size, uint8_t* status) {
  if (!file || !count || !status || (cap && (!handle_off || !handle_size)))
    return lgs::set_error(LGS_EINVAL, "NULL argument");
  if (filter_name && (!filter_off || !filter_size))
    return lgs::set_error(LGS_EINVAL, "NULL filter handle output");
  *count = 0;
  *status = LGS_ST_OK;
  if (filter_off) *filter_off = ~0ull;
  if (filter_size) *filter_size = 0;
  if (key_off) key_off[0] = 0;
  // Footer (table.c:127-145, format.c:116-137).
  if (file_len < kFooterSize) {
    *status = LGS_ST_CORRUPT;                             // "file is too short"
    return LGS_OK;
  }
  const uint8_t* f = file + file_len - kFooterSize;
  uint64_t magic = 0;
  for (int i = 7; i >= 0; --i) magic = (magic << 8) | f[kFooterSize - 8 + i];
  uint64_t mi_off = 0, mi_size = 0, ix_off = 0, ix_size = 0;
  const uint8_t* p = f;
  size_t n = kFooterSize;
  if (magic != kTableMagic || !varint64(&mi_off, &p, &n) || !varint64(&mi_size, &p, &n) ||
      !varint64(&ix_off, &p, &n) || !varint64(&ix_size, &p, &n)) {
    *status = LGS_ST_CORRUPT;
    return LGS_OK;
  }
  // Index block (table.c:148-158).
  std::vector<uint8_t> blk;
  uint8_t st = 0;
  int rc = read_block(file, file_len, ix_off, ix_size, paranoid_checks != 0, &blk, &st);
  if (rc != LGS_OK) return rc;
  if (st != LGS_ST_OK) {
    *status = st;
    return LGS_OK;
  }
  // Its entries (two_level_iterator.c: one data block per entry).  A value
  // that is no handle is skipped with the table's status set to corruption
  // (the two-level iterator's "bad block handle"); a bad entry ends the walk.
  uint32_t cnt = 0;
  size_t kat = 0;
  bool overflow = false, bad_handle = false;
  const uint8_t walk = walk_block(blk, internal_keys != 0,
                                  [&](const std::string& k, const uint8_t* v, size_t vn) {
    uint64_t o, s;
    if (!handle_import(&o, &s, v, vn)) {
      bad_handle = true;
      return;
    }
    if (cnt >= cap || (keys && kat + k.size() > keys_cap)) {
      overflow = true;
      return;
    }
    handle_off[cnt] = o;
    handle_size[cnt] = s;
    if (keys) {
      memcpy(keys + kat, k.data(), k.size());
      kat += k.size();
    }
    ++cnt;
    if (key_off) key_off[cnt] = kat;
  });
  *count = cnt;
  if (overflow)
    return lgs::set_error(LGS_ENOSPC, "more index entries than cap / keys_cap");
  *status = walk != LGS_ST_OK ? walk : (bad_handle ? (uint8_t)LGS_ST_CORRUPT : (uint8_t)LGS_ST_OK);
  // Filter handle: metaindex entry `filter_name` (table.c:78-120; errors there
  // are not propagated, :103-106).  The metaindex is sorted: the seek's hit is
  // the first key >= name, a match only if equal.
  if (filter_name) {
    rc = read_block(file, file_len, mi_off, mi_size, paranoid_checks != 0, &blk, &st);
    if (rc != LGS_OK) return rc;
    if (st == LGS_ST_OK) {
      const std::string name(filter_name);
      bool done = false;
      walk_block(blk, false, [&](const std::string& k, const uint8_t* v, size_t vn) {
        if (done || k < name) return;
        done = true;
        uint64_t o, s;
        if (k == name && handle_import(&o, &s, v, vn)) {
          *filter_off = o;
          *filter_size = s;
        }
      });
    }
  }
  return LGS_OK;
}
