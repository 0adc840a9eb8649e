// step_kernels.hip — the fused step kernels (k_step, ps_env.h) of one
// (task, control) pair: built once per pair with -DPS_STEP_TASK=t
// -DPS_STEP_CONTROL=c (pandasim/build.py), so the twelve pairs compile as
// parallel jobs.  ps_step (pandasim.hip) calls the pair's launcher.
#include "ps_env.h"

#if !defined(PS_STEP_TASK) || !defined(PS_STEP_CONTROL)
#error "build with -DPS_STEP_TASK=<task> -DPS_STEP_CONTROL=<control>"
#endif

int PS_STEP_LAUNCHER_NAME(PS_STEP_TASK, PS_STEP_CONTROL)(ps_ctx *c, void *state, const ps_step_io &io, int lanes,
                                                         hipStream_t st) {
    constexpr int T = PS_STEP_TASK, C = PS_STEP_CONTROL;
    KParams P = params_of(c, state);
    P.autoreset = io.autoreset;
    P.nonfinite = c->nonfinite;
    P.reset_nonfinite = c->reset_nonfinite;
    // the gain rows belong to a state buffer: another buffer than the one the
    // last step wrote (a swapped or copied-in state) gets them written too
    P.write_gains = c->gains_dirty || state != c->gains_state;
    const dim3 g = grid_of(P.n * lanes, kBlock), b(kBlock);
#define PS_LAUNCH(G)                                                                                               \
    hipLaunchKernelGGL((k_step<T, C, G>), g, b, 0, st, P, io.actions, io.obs, io.ag, io.dg, io.reward,             \
                       io.terminated, io.truncated, io.final_obs, io.final_ag)
    // groups of 16 or 8 lanes per env exist for the one-object and robot-only tasks
    if constexpr (T != PS_TASK_STACK) {
        if (lanes == 16) PS_LAUNCH(16);
        else if (lanes == 8) PS_LAUNCH(8);
        else PS_LAUNCH(1);
    } else {
        PS_LAUNCH(1);
    }
#undef PS_LAUNCH
    return check_launch(c);
}

