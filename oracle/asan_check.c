/*
 * asan_check.c -- TEST INFRASTRUCTURE ONLY (sanitizers).
 *
 * Drives every public entry point of the oracle (panda_oracle.c) through all
 * six tasks and both control modes -- seeded resets, random-action steps with
 * auto-reset, engine substeps, inverse kinematics, link/base queries and the
 * task layer -- so that `make asan` (AddressSanitizer + UndefinedBehavior
 * Sanitizer, any report fatal) checks the restatement for out-of-bounds
 * accesses, use of uninitialised stack rows and undefined arithmetic.
 * Exit status 0 = clean.
 */
#include <stdio.h>
#include <string.h>

#include "panda_oracle.h"

static uint64_t lcg = 0x9E3779B97F4A7C15ULL;
static float uniform_pm1(void) {
    lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL;
    return (float)((lcg >> 40) * (2.0 / 16777216.0) - 1.0);
}

int main(void) {
    int checked = 0;
    for (int task = 0; task < 6; task++)
        for (int control = 0; control < 2; control++) {
            po_config cfg;
            po_default_config(&cfg, task, control, control);
            po_env envs[3];
            float obs[32], ag[8], dg[8], fo[32], fa[8], r;
            uint8_t te, tr;
            po_stats st;
            memset(&st, 0, sizeof st);
            for (int e = 0; e < 3; e++) {
                po_init_env(&cfg, &envs[e]);
                po_reset(&cfg, &envs[e], 1, 1000 + 17 * task + e, obs, ag, dg);
            }
            int na = po_action_dim(&cfg);
            for (int s = 0; s < 60; s++)
                for (int e = 0; e < 3; e++) {
                    float a[8];
                    for (int k = 0; k < na; k++) a[k] = uniform_pm1() * 1.2f; /* includes clipped values */
                    po_step(&cfg, &envs[e], a, obs, ag, dg, &r, &te, &tr, 1, fo, fa, &st);
                    checked++;
                }
            double pos[3], quat[4], lv[3], av[3], q[9], M[81], h[9];
            po_link_state(&cfg, &envs[0], 11, pos, quat, lv, av);
            double tgt[3] = {pos[0] + 0.02, pos[1] - 0.02, pos[2] + 0.01}, orn[4] = {1, 0, 0, 0};
            po_inverse_kinematics(&cfg, envs[0].q, 11, tgt, orn, q);
            po_mass_matrix(&cfg, envs[0].q, M);
            po_bias_forces(&cfg, envs[0].q, envs[0].qd, h);
            po_sim_step(&cfg, &envs[1], &st);
            po_get_obs(&cfg, &envs[2], obs, ag, dg);
            (void)po_compute_reward(task, control, ag, envs[2].goal);
            (void)po_is_success(task, ag, envs[2].goal);
            double rpy[3];
            po_euler_from_quaternion(envs[2].obj[0].quat, rpy);
        }
    printf("asan_check: %d env steps over 6 tasks x 2 controls clean\n", checked);
    return 0;
}
