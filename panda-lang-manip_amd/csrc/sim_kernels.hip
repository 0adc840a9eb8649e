// sim_kernels.hip — the plugin path's substep kernel (k_sim_step, ps_env.h)
// of one scene: built once per (objects, shape) with -DPS_SIM_NOBJ=n
// -DPS_SIM_SHAPE=s (pandasim/build.py).  ps_sim_step (pandasim.hip) calls it.
#include "ps_env.h"

#if !defined(PS_SIM_NOBJ) || !defined(PS_SIM_SHAPE)
#error "build with -DPS_SIM_NOBJ=<objects> -DPS_SIM_SHAPE=<shape>"
#endif

int PS_SIM_LAUNCHER_NAME(PS_SIM_NOBJ, PS_SIM_SHAPE)(ps_ctx *c, void *state, int n_substeps, hipStream_t st) {
    KParams P = params_of(c, state);
    hipLaunchKernelGGL((k_sim_step<PS_SIM_NOBJ, PS_SIM_SHAPE>), grid_of(P.n, kBlock), dim3(kBlock), 0, st, P,
                       n_substeps);
    return check_launch(c);
}
