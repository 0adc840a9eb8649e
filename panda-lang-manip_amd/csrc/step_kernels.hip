// step_kernels.hip — the fused step kernels (k_step, ps_env.h) of one
// (task, control) pair: built once per pair with -DPS_STEP_TASK=t
// -DPS_STEP_CONTROL=c (pandasim/build.py), so the pairs compile as parallel
// jobs.  ps_step (pandasim.hip) calls the pair's launcher.  The one-lane
// kernel and the launcher form one object; the 16- and 8-lane group kernels
// form a second (-DPS_STEP_GROUPS=1), compiled with the same flags (-O3;
// DESIGN.md §12.6).
#include "ps_env.h"

#ifdef PS_EXPERIMENT_G2
#define PS_G2_ENABLED 1
#else
#define PS_G2_ENABLED 0
#endif

#if !defined(PS_STEP_TASK) || !defined(PS_STEP_CONTROL)
#error "build with -DPS_STEP_TASK=<task> -DPS_STEP_CONTROL=<control>"
#endif

#define PS_LAUNCH(G)                                                                                               \
    hipLaunchKernelGGL((k_step<PS_STEP_TASK, PS_STEP_CONTROL, G>), grid_of(P.n * (G), kBlock), dim3(kBlock), 0, st, \
                       P, io.actions, io.obs, io.ag, io.dg, io.reward, io.terminated, io.truncated, io.final_obs,  \
                       io.final_ag)

#if defined(PS_STEP_GROUPS) && PS_STEP_GROUPS
static_assert(PS_STEP_TASK != PS_TASK_STACK, "Stack has no group kernels (two objects: 21 DoFs)");

int PS_STEP_GROUP_LAUNCHER_NAME(PS_STEP_TASK, PS_STEP_CONTROL)(ps_ctx *c, const void *params, const ps_step_io &io,
                                                               int lanes, hipStream_t st) {
    const KParams P = *static_cast<const KParams *>(params);
#ifdef PS_EXPERIMENT_G2
    // two lanes per env, a measured experiment only
    if (lanes == 2) {
        PS_LAUNCH(2);
        return check_launch(c);
    }
#endif
    if (lanes == 16) PS_LAUNCH(16);
    else PS_LAUNCH(8);
    return check_launch(c);
}

#else
int PS_STEP_LAUNCHER_NAME(PS_STEP_TASK, PS_STEP_CONTROL)(ps_ctx *c, void *state, const ps_step_io &io, int lanes,
                                                         hipStream_t st) {
    KParams P = params_of(c, state);
    P.autoreset = io.autoreset;
    P.nonfinite = c->nonfinite;
    P.reset_nonfinite = c->reset_nonfinite;
    // the gain rows belong to a state buffer: another buffer than the one the
    // last step wrote (a swapped or copied-in state) gets them written too
    P.write_gains = c->gains_dirty || state != c->gains_state;
    // groups of 16 or 8 lanes per env exist for the one-object and robot-only tasks
#if PS_STEP_TASK != 4  // PS_TASK_STACK
    if (lanes == 16 || lanes == 8 || (PS_G2_ENABLED && lanes == 2))
        return PS_STEP_GROUP_LAUNCHER_NAME(PS_STEP_TASK, PS_STEP_CONTROL)(c, &P, io, lanes, st);
#endif
    PS_LAUNCH(1);
    return check_launch(c);
}
#endif
#undef PS_LAUNCH
