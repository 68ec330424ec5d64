// qp_medium.hip — placeholder for the n > 16 kernel family (filled in below the small kernels).
#include "qp_common.h"

extern "C" hipError_t qpk_launch_medium(const qpk::QpArgs*, hipStream_t, int* handled,
                                        const char**) {
  *handled = 0;
  return hipSuccess;
}
extern "C" const char* qpk_medium_name(int, int, int) { return nullptr; }
extern "C" int qpk_medium_max_n(void) { return 0; }
extern "C" int qpk_medium_max_m(void) { return 0; }
