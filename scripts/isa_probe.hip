// ISA probe (compiled with -S only, never launched): the box-cylinder pick of
// Slide's gripper candidates in a kernel of its own, so its instruction count
// can be read off the assembly (scripts/isa_count.sh)
#include "ps_env.h"

__global__ void probe_boxcyl_pick(const float *in, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float *p = in + i * 40;
    Scene sc{};
    sc.half = mk(p[0], p[0], p[1]);
    const V3 xc = mk(p[2], p[3], p[4]), yc = mk(p[5], p[6], p[7]), xh = mk(p[8], p[9], p[10]);
    M3 xR, yR;
    for (int q = 0; q < 9; q++) { xR.m[q] = p[11 + q]; yR.m[q] = p[20 + q]; }
    const V3 w = mk(p[29], p[30], p[31]);
    RCand c0, c1;
    const BoxCyl bcy(sc, xc, xR, xh, yc, yR);
    const int ns = bcy.pick(sc, xc, w, c0, c1);
    float *o = out + i * 21;
    const float v[21] = {c0.pA.x, c0.pA.y, c0.pA.z, c0.pB.x, c0.pB.y, c0.pB.z, c0.n.x, c0.n.y, c0.n.z, c0.dist,
                         c1.pA.x, c1.pA.y, c1.pA.z, c1.pB.x, c1.pB.y, c1.pB.z, c1.n.x, c1.n.y, c1.n.z, c1.dist, (float)ns};
    for (int q = 0; q < 21; q++) o[q] = v[q];
}

// the box-cube pick of the Push/PickAndPlace/Flip gripper candidates
__global__ void probe_boxcube_pick(const float *in, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float *p = in + i * 40;
    const V3 xc = mk(p[2], p[3], p[4]), yc = mk(p[5], p[6], p[7]), xh = mk(p[8], p[9], p[10]);
    const V3 yh = mk(p[0], p[0], p[0]);
    M3 xR, yR;
    for (int q = 0; q < 9; q++) { xR.m[q] = p[11 + q]; yR.m[q] = p[20 + q]; }
    const V3 w = mk(p[29], p[30], p[31]);
    RCand c0, c1;
    const BoxCube bcu(xc, xR, xh, yc, yR, yh);
    const int ns = bcu.pick(xc, w, c0, c1);
    float *o = out + i * 21;
    const float v[21] = {c0.pA.x, c0.pA.y, c0.pA.z, c0.pB.x, c0.pB.y, c0.pB.z, c0.n.x, c0.n.y, c0.n.z, c0.dist,
                         c1.pA.x, c1.pA.y, c1.pA.z, c1.pB.x, c1.pB.y, c1.pB.z, c1.n.x, c1.n.y, c1.n.z, c1.dist, (float)ns};
    for (int q = 0; q < 21; q++) o[q] = v[q];
}
