// ps_task.h — device restatement of the task layer:
//   numpy SeedSequence + PCG64 + Generator.uniform (gymnasium seeding,
//   panda_gym/envs/core.py:244), goal/object sampling (reach.py:47-54,
//   push.py:69-87, pick_and_place.py:65-85), the fp64 distance / success /
//   reward (utils.py:4-15, push.py:89-98) and getEulerFromQuaternion.
// Integer work is exact; the fp64 arithmetic uses explicit round-to-nearest
// intrinsics (no FMA contraction) so results are bit-identical to numpy.
#pragma once

#include "ps_common.h"

namespace ps {

struct Pcg {
    uint64_t sh, sl, ih, il;  // state hi/lo, increment hi/lo
};

PS_D void pcg_step(Pcg &r) {
    const uint64_t MH = 0x2360ED051FC65DA4ULL, ML = 0x4385DF649FCCF645ULL;
    uint64_t lo = r.sl * ML;
    uint64_t hi = __umul64hi(r.sl, ML) + r.sl * MH + r.sh * ML;
    uint64_t nl = lo + r.il;
    uint64_t carry = nl < lo ? 1ULL : 0ULL;
    r.sh = hi + r.ih + carry;
    r.sl = nl;
}

PS_D uint64_t pcg_next(Pcg &r) {
    pcg_step(r);
    uint64_t x = r.sh ^ r.sl;
    unsigned rot = (unsigned)(r.sh >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

// Opaque barriers: hipcc contracts a*b+c into an FMA across inlined helper
// calls even under `#pragma clang fp contract(off)`; numpy rounds the product
// first.  An empty asm on the product keeps it a separate, rounded value.
PS_D double opaque(double x) {
    asm volatile("" : "+v"(x));
    return x;
}
PS_D float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

PS_D double pcg_double(Pcg &r) { return __dmul_rn((double)(pcg_next(r) >> 11), 1.0 / 9007199254740992.0); }

// Generator.uniform: low + (high - low) * next_double
PS_D double uniform(Pcg &r, double lo, double hi) {
#pragma clang fp contract(off)
    double range = __dsub_rn(hi, lo);
    double u = pcg_double(r);
    return __dadd_rn(lo, opaque(__dmul_rn(range, u)));
}

// SeedSequence(seed).generate_state(4, uint64) -> pcg64_set_seed
PS_D Pcg pcg_seed(uint64_t seed) {
    const uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
    const uint32_t MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
    uint32_t e0 = (uint32_t)seed, e1 = (uint32_t)(seed >> 32);
    int nent = (seed >> 32) ? 2 : 1;
    uint32_t pool[4], hc = INIT_A;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t v = (i == 0 ? e0 : (i == 1 && nent == 2 ? e1 : 0u)) ^ hc;
        hc *= MULT_A;
        v *= hc;
        v ^= v >> 16;
        pool[i] = v;
    }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int d = 0; d < 4; d++)
            if (s != d) {
                uint32_t v = pool[s] ^ hc;
                hc *= MULT_A;
                v *= hc;
                v ^= v >> 16;
                uint32_t r = MIX_L * pool[d] - MIX_R * v;
                r ^= r >> 16;
                pool[d] = r;
            }
    uint32_t w[8], hb = INIT_B;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3] ^ hb;
        hb *= MULT_B;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
    Pcg r;
    // inc = (initseq << 1) | 1 with initseq = v2:v3
    r.ih = (v2 << 1) | (v3 >> 63);
    r.il = (v3 << 1) | 1ULL;
    r.sh = 0;
    r.sl = 0;
    pcg_step(r);
    // state += initstate (v0:v1)
    uint64_t nl = r.sl + v1;
    r.sh = r.sh + v0 + (nl < r.sl ? 1ULL : 0ULL);
    r.sl = nl;
    pcg_step(r);
    return r;
}

// d = || float(ag) - goal ||_2 in fp64, summed left to right as numpy does
PS_D double goal_distance(float a0, float a1, float a2, double g0, double g1, double g2) {
#pragma clang fp contract(off)
    double d0 = __dsub_rn((double)a0, g0), d1 = __dsub_rn((double)a1, g1), d2 = __dsub_rn((double)a2, g2);
    double s = opaque(__dmul_rn(d0, d0));
    s = __dadd_rn(s, opaque(__dmul_rn(d1, d1)));
    s = __dadd_rn(s, opaque(__dmul_rn(d2, d2)));
    return __dsqrt_rn(s);
}

PS_D double goal_distance_f64(double a0, double a1, double a2, double g0, double g1, double g2) {
#pragma clang fp contract(off)
    double d0 = __dsub_rn(a0, g0), d1 = __dsub_rn(a1, g1), d2 = __dsub_rn(a2, g2);
    double s = opaque(__dmul_rn(d0, d0));
    s = __dadd_rn(s, opaque(__dmul_rn(d1, d1)));
    s = __dadd_rn(s, opaque(__dmul_rn(d2, d2)));
    return __dsqrt_rn(s);
}

PS_D float reward_of(int reward_type, double d) {
    if (reward_type == 0) return d > PM_DISTANCE_THRESHOLD ? -1.0f : -0.0f;
    return -__double2float_rn(d);
}

// all-float32 operands: numpy keeps the arithmetic and the comparison with the
// Python-float threshold in float32 (the threshold becomes 0.05f)
PS_D float goal_distance_f32(float a0, float a1, float a2, float g0, float g1, float g2) {
#pragma clang fp contract(off)
    float d0 = __fsub_rn(a0, g0), d1 = __fsub_rn(a1, g1), d2 = __fsub_rn(a2, g2);
    float s = opaque(__fmul_rn(d0, d0));
    s = __fadd_rn(s, opaque(__fmul_rn(d1, d1)));
    s = __fadd_rn(s, opaque(__fmul_rn(d2, d2)));
    // correctly rounded fp32 sqrt: the fp64 root rounded once to fp32 is
    // exact-rounded for sqrt (53 >= 2*24 + 2); v_sqrt_f32 alone is not
    return __double2float_rn(__dsqrt_rn((double)s));
}

PS_D float reward_of_f32(int reward_type, float d) {
    if (reward_type == 0) return d > (float)PM_DISTANCE_THRESHOLD ? -1.0f : -0.0f;
    return -d;
}

// getEulerFromQuaternion (fp32)
PS_D V3 euler_from_quat(Q4 q) {
    float sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    float sarg = -2.0f * (q.x * q.z - q.w * q.y);
    if (sarg <= -0.99999f) return mk(0.0f, -0.5f * 3.14159265358979323846f, 2.0f * atan2f(q.x, -q.y));
    if (sarg >= 0.99999f) return mk(0.0f, 0.5f * 3.14159265358979323846f, 2.0f * atan2f(-q.x, q.y));
    return mk(atan2f(2.0f * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz), asinf(sarg),
              atan2f(2.0f * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz));
}

}  // namespace ps
