// lgs_encode_service.hip -- the drop-in service's encode kernel
// (encode_service_kernel, lgs_encode.hip) in a compilation of its own: the
// batch encode kernels are built with the max-ILP machine scheduler, which
// lengthens one resident wave's walk of a block (build.py).
#define LGS_ENCODE_SERVICE_ONLY
#include "lgs_encode.hip"
