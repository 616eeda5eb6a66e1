// drb_step_inst.hip -- one instantiation of the step kernel (drb_step.hpp)
// and its launcher, compiled once per (R, kind) with -DDRB_INST_R and
// -DDRB_INST_KIND (dragonboat_amd/build.py).  The 80 instantiations (the
// lean kernel of drb_lean.hpp and the LOCAL kinds among them) are
// independent translation units so the build runs them in parallel; the
// engine (drb_engine.hip) calls them through kStepLaunch (drb_launch.hpp).
//
// Written for gfx950 (MI355X) only.
#include <hip/hip_runtime.h>

#include "drb_launch.hpp"
#include "drb_step.hpp"

#ifndef DRB_INST_R
#error "DRB_INST_R (replicas per group) is required"
#endif
#ifndef DRB_INST_KIND
#error "DRB_INST_KIND (drb_launch.hpp StepKind) is required"
#endif

namespace drb {

void DRB_STEP_LAUNCH_NAME(DRB_INST_R, DRB_INST_KIND)(const View &v,
                                                     const RoundParams &p,
                                                     unsigned grid,
                                                     hipStream_t s) {
  constexpr int K = DRB_INST_KIND;
  if constexpr (K == SK_LEAD_LEAN || K == SK_FOLLOW_LEAN) {
    lean_kernel<DRB_INST_R, K == SK_LEAD_LEAN><<<grid, 256, 0, s>>>(v, p);
  } else {
    constexpr bool LOCAL = K >= SK_LEAD_LOCAL;  // (kinds 9-12: 0-3 LOCAL)
    constexpr int B = LOCAL ? (K == SK_LEAD_LOCAL       ? SK_LEAD
                               : K == SK_FOLLOW_LOCAL   ? SK_FOLLOW
                               : K == SK_LEAD_EXT_LOCAL ? SK_LEAD_EXT
                                                        : SK_FOLLOW_EXT)
                            : K;
    constexpr bool LEAD =
        B == SK_LEAD || B == SK_LEAD_EXT || B == SK_SLOW || B == SK_LEAD_FWD;
    constexpr bool FWD =
        B == SK_SLOW || B == SK_LEAD_FWD || B == SK_FOLLOW_FWD;
    constexpr bool EXT = B == SK_LEAD_EXT || B == SK_FOLLOW_EXT || FWD;
    constexpr bool SLOW = B == SK_SLOW;
    // the leader's per-remote entry-row floors (LDS) exist with placement C4
    const size_t dyn =
        LEAD && !LOCAL && v.remote_mask ? DRB_INST_R * 256 * 8 : 0;
    step_kernel<DRB_INST_R, LEAD, EXT, SLOW, FWD, LOCAL>
        <<<grid, 256, dyn, s>>>(v, p);
  }
}

}  // namespace drb
