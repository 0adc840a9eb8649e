// calib_fetch.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the
// access width the step kernel uses (one 4-byte word per lane, consecutive
// lanes on consecutive words: the SoA row pattern of k_step).
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for 16-B-per-lane
// streams; this measures the factor for 4-B-per-lane ones.
//
//   k_read : reads a 1 GiB buffer once (beyond the 256 MiB Infinity Cache)
//   k_write: writes a 1 GiB buffer once
// Run it under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` and `--pmc
// WRITE_SIZE`; the known byte count is printed as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_read(const float *__restrict__ x, int64_t n, float *out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float s = 0.0f;
    for (; i < n; i += stride) s += x[i];
    if (s == 12345.678f) out[0] = s;  // keeps the loads alive, never true for zeros
}

__global__ __launch_bounds__(256) void k_write(float *__restrict__ x, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) x[i] = (float)(i & 7);
}

int main() {
    const int64_t n = (int64_t)1 << 28;  // 1 GiB of floats
    float *x, *out;
    if (hipMalloc(&x, n * 4) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(x, 0, n * 4);
    (void)hipDeviceSynchronize();
    const int grid = 256 * 32;
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, x, n, out);
        hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, x, n);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"read_bytes_per_launch\": %lld, \"write_bytes_per_launch\": %lld}\n", (long long)(n * 4),
           (long long)(n * 4));
    (void)hipFree(x);
    (void)hipFree(out);
    return 0;
}
