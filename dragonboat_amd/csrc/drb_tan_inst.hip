// drb_tan_inst.hip -- the tan record kernels (drb_tan.hpp) and their
// launchers, compiled twice (dragonboat_amd/build.py): DRB_TAN_KERNELS=1
// the select pass and the multiplexed chain, =2 the write pass.  Their
// register allocation is the longest part of the build, so they are
// translation units of their own.
//
// Written for gfx950 (MI355X) only.
#include <hip/hip_runtime.h>

#include "drb_launch.hpp"
#include "drb_tan.hpp"

namespace drb {

#if DRB_TAN_KERNELS == 1
void tan_launch_select(const View &v, uint32_t round, uint64_t max_log,
                       uint32_t *list, uint32_t per_list, uint32_t *n,
                       unsigned blocks, hipStream_t s) {
  k_tan_select<<<blocks, 256, 0, s>>>(v, round, max_log, list, per_list, n);
}

void tan_launch_chain(const View &v, uint64_t max_log, unsigned blocks,
                      hipStream_t s) {
  k_tanm_chain<<<blocks, 64, 0, s>>>(v, max_log);
}
#elif DRB_TAN_KERNELS == 2
void tan_launch_write(const View &v, uint32_t round, uint64_t max_log,
                      const uint32_t *list, uint32_t per_list,
                      const uint32_t *n, unsigned blocks, hipStream_t s) {
  k_tan_write<<<blocks, 256, 0, s>>>(v, round, max_log, list, per_list, n);
}
#else
#error "DRB_TAN_KERNELS must be 1 or 2"
#endif

}  // namespace drb
