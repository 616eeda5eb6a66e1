// drb_launch.hpp -- the step kernel's instantiations as separately compiled
// launchers (drb_step_inst.hip), one per (replicas per group, kind).
#pragma once
#include <hip/hip_runtime.h>

#include "drb_layout.hpp"

namespace drb {

struct RoundParams;  // drb_step.hpp

enum StepKind : int {
  SK_LEAD = 0,        // step_kernel<R, true, false>: leaders, C3 paths
  SK_LEAD_EXT = 1,    // step_kernel<R, true, true>: + long Cmds, out-of-line
                      //   values, EntryBatch / tan encoding, Quiesce
  SK_FOLLOW = 2,      // step_kernel<R, false, false>
  SK_FOLLOW_EXT = 3,  // step_kernel<R, false, true>
  SK_SLOW = 4,        // step_kernel<R, true, true, true>: the raft launch
  SK_LEAD_FWD = 5,    // step_kernel<R, true, true, false, true>: EXT with
                      //   forwarded proposals (drb_config.forward_proposals)
  SK_FOLLOW_FWD = 6,  // step_kernel<R, false, true, false, true>
  SK_LEAD_LEAN = 7,   // lean_kernel<R, true>: a listed round's heartbeat-
                      //   only leaders (drb_lean.hpp)
  SK_FOLLOW_LEAN = 8,  // lean_kernel<R, false>
  // the LOCAL instantiations of kinds 0-3 (no remote planes compiled in:
  // engines without placement, View.remote_mask 0), built for R = 3 and 5;
  // other R run the kinds they stand for
  SK_LEAD_LOCAL = 9,
  SK_FOLLOW_LOCAL = 10,
  SK_LEAD_EXT_LOCAL = 11,
  SK_FOLLOW_EXT_LOCAL = 12,
  NUM_STEP_KINDS
};

typedef void (*StepLaunchFn)(const View &v, const RoundParams &p,
                             unsigned grid, hipStream_t s);

#define DRB_STEP_LAUNCH_NAME2(R, K) step_launch_r##R##_k##K
#define DRB_STEP_LAUNCH_NAME(R, K) DRB_STEP_LAUNCH_NAME2(R, K)

#define DRB_DECLARE_STEP_LAUNCH(R, K)                                      \
  void DRB_STEP_LAUNCH_NAME(R, K)(const View &v, const RoundParams &p,     \
                                  unsigned grid, hipStream_t s);
#define DRB_DECLARE_STEP_LAUNCH_R(R)                                      \
  DRB_DECLARE_STEP_LAUNCH(R, 0)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 1)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 2)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 3)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 4)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 5)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 6)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 7)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 8)
DRB_DECLARE_STEP_LAUNCH_R(1)
DRB_DECLARE_STEP_LAUNCH_R(2)
DRB_DECLARE_STEP_LAUNCH_R(3)
DRB_DECLARE_STEP_LAUNCH_R(4)
DRB_DECLARE_STEP_LAUNCH_R(5)
DRB_DECLARE_STEP_LAUNCH_R(6)
DRB_DECLARE_STEP_LAUNCH_R(7)
DRB_DECLARE_STEP_LAUNCH_R(8)
#define DRB_DECLARE_STEP_LAUNCH_LOCAL(R)                                  \
  DRB_DECLARE_STEP_LAUNCH(R, 9)                                           \
  DRB_DECLARE_STEP_LAUNCH(R, 10)                                          \
  DRB_DECLARE_STEP_LAUNCH(R, 11)                                          \
  DRB_DECLARE_STEP_LAUNCH(R, 12)
DRB_DECLARE_STEP_LAUNCH_LOCAL(3)
DRB_DECLARE_STEP_LAUNCH_LOCAL(5)

// the tan record kernels (drb_tan.hpp), compiled in drb_tan_inst.hip
void tan_launch_select(const View &v, uint32_t round, uint64_t max_log,
                       uint32_t *list, uint32_t per_list, uint32_t *n,
                       unsigned blocks, hipStream_t s);
void tan_launch_chain(const View &v, uint64_t max_log, unsigned blocks,
                      hipStream_t s);
void tan_launch_write(const View &v, uint32_t round, uint64_t max_log,
                      const uint32_t *list, uint32_t per_list,
                      const uint32_t *n, unsigned blocks, hipStream_t s);

#ifndef DRB_INST_R
// kStepLaunch[R - 1][kind]
#define DRB_STEP_LAUNCH_ROW(R)                                            \
  {DRB_STEP_LAUNCH_NAME(R, 0), DRB_STEP_LAUNCH_NAME(R, 1),                \
   DRB_STEP_LAUNCH_NAME(R, 2), DRB_STEP_LAUNCH_NAME(R, 3),                \
   DRB_STEP_LAUNCH_NAME(R, 4), DRB_STEP_LAUNCH_NAME(R, 5),                \
   DRB_STEP_LAUNCH_NAME(R, 6), DRB_STEP_LAUNCH_NAME(R, 7),                \
   DRB_STEP_LAUNCH_NAME(R, 8), DRB_STEP_LAUNCH_NAME(R, 0),                \
   DRB_STEP_LAUNCH_NAME(R, 2), DRB_STEP_LAUNCH_NAME(R, 1),                \
   DRB_STEP_LAUNCH_NAME(R, 3)}
#define DRB_STEP_LAUNCH_ROW_LOCAL(R)                                      \
  {DRB_STEP_LAUNCH_NAME(R, 0), DRB_STEP_LAUNCH_NAME(R, 1),                \
   DRB_STEP_LAUNCH_NAME(R, 2), DRB_STEP_LAUNCH_NAME(R, 3),                \
   DRB_STEP_LAUNCH_NAME(R, 4), DRB_STEP_LAUNCH_NAME(R, 5),                \
   DRB_STEP_LAUNCH_NAME(R, 6), DRB_STEP_LAUNCH_NAME(R, 7),                \
   DRB_STEP_LAUNCH_NAME(R, 8), DRB_STEP_LAUNCH_NAME(R, 9),                \
   DRB_STEP_LAUNCH_NAME(R, 10), DRB_STEP_LAUNCH_NAME(R, 11),              \
   DRB_STEP_LAUNCH_NAME(R, 12)}
static const StepLaunchFn kStepLaunch[8][NUM_STEP_KINDS] = {
    DRB_STEP_LAUNCH_ROW(1),       DRB_STEP_LAUNCH_ROW(2),
    DRB_STEP_LAUNCH_ROW_LOCAL(3), DRB_STEP_LAUNCH_ROW(4),
    DRB_STEP_LAUNCH_ROW_LOCAL(5), DRB_STEP_LAUNCH_ROW(6),
    DRB_STEP_LAUNCH_ROW(7),       DRB_STEP_LAUNCH_ROW(8)};
#endif

}  // namespace drb
