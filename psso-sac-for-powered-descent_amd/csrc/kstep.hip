// kstep.hip -- explicit instantiations of the step kernel's launchers (pd_step_impl.h) for one
// (precision, phase family, wind) triple, chosen by -DPD_KR (0 double, 1 float), -DPD_KPH
// (0 pure throttle, 1 landing_burn, 2 the other phases) and -DPD_KW (0/1).  pdenv/build.py
// compiles this file once per triple, in parallel, and links the objects into libpdenv.so.
#include "pd_step_impl.h"

#if !defined(PD_KR) || !defined(PD_KPH) || !defined(PD_KW)
#error "kstep.hip needs -DPD_KR=0|1 -DPD_KPH=0|1|2 -DPD_KW=0|1"
#endif

namespace pd {
#if PD_KR == 0
using KR = double;
#else
using KR = float;
#endif
constexpr bool KW = PD_KW != 0;

#define PD_INST_STEP(RT)                                                          \
    template void launch_step<KR, PD_KPH, RT, KW, 1>(const StepArgs<KR>&, hipStream_t);  \
    template void launch_step<KR, PD_KPH, RT, KW, 2>(const StepArgs<KR>&, hipStream_t);  \
    template void launch_step<KR, PD_KPH, RT, KW, 4>(const StepArgs<KR>&, hipStream_t);  \
    template void launch_step<KR, PD_KPH, RT, KW, 8>(const StepArgs<KR>&, hipStream_t);  \
    template void launch_step<KR, PD_KPH, RT, KW, 16>(const StepArgs<KR>&, hipStream_t);

// RL and PD_RTD_NONE share the RL instantiation; PSO exists for the two landing burns, with the
// policy-rollout (fused actor) kernels.  -DPD_KLPE=n (experiments): the RL kernel at n lanes only.
#if defined(PD_KRK4)
// the non-parity RK4 mode (pure throttle, no wind; -DPD_KPH=0 -DPD_KW=0): LPE 2 and 16
static_assert(PD_KPH == 0 && PD_KW == 0, "RK4 unit: pure throttle without wind");
template void launch_step<KR, 0, 0, false, 2, true>(const StepArgs<KR>&, hipStream_t);
template void launch_step<KR, 0, 0, false, 16, true>(const StepArgs<KR>&, hipStream_t);
template void launch_step<KR, 0, 1, false, 2, true>(const StepArgs<KR>&, hipStream_t);
template void launch_step<KR, 0, 1, false, 16, true>(const StepArgs<KR>&, hipStream_t);
#elif defined(PD_KLPE)
template void launch_step<KR, PD_KPH, 0, KW, PD_KLPE>(const StepArgs<KR>&, hipStream_t);
#else
PD_INST_STEP(0)
#endif
#if PD_KPH < 2 && !defined(PD_KLPE) && !defined(PD_KRK4)
PD_INST_STEP(1)
// (policy rollouts run at 2 lanes per env: the per-lane actor + the LPE 2 table path fit the
// register file without scratch, which the LPE 4/8 variants did not)
template void launch_policy_lpe<KR, PD_KPH, KW, 2>(const StepArgs<KR>&, int64_t, hipStream_t);
// (LPE 4/8: the lanes-per-env sweep of the policy rollouts, PDENV_PLPE)
template void launch_policy_lpe<KR, PD_KPH, KW, 4>(const StepArgs<KR>&, int64_t, hipStream_t);
template void launch_policy_lpe<KR, PD_KPH, KW, 8>(const StepArgs<KR>&, int64_t, hipStream_t);
#endif
}  // namespace pd
