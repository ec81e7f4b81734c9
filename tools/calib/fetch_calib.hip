// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the step kernel's access widths
// (MI355X_MICROARCH.md, HBM: only 16-B-per-lane streaming reads are calibrated there).
// Each kernel streams N elements once, coalesced, lane i -> element i, at 4 B (dword),
// 8 B (dwordx2, the fp64 goal) and 16 B per lane; the known byte counts are printed so the
// PMC pass can be divided by them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <class T>
__global__ __launch_bounds__(256) void copy_kernel(const T* __restrict__ a, T* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

/* the step kernel's pattern: SoA rows [K][N], 4 envs per wave (16 lanes each),
 * the lead lane of an env loads / stores one dword per row, blocks dealt to XCDs as xcd_block */
__global__ __launch_bounds__(64) void soa_kernel(const float* __restrict__ a, float* __restrict__ b, int n, int k) {
    const int nb = gridDim.x, bb = blockIdx.x;
    const int blk = (nb % 8) ? bb : (bb % 8) * (nb / 8) + bb / 8;
    const int env = blk * 4 + (int)threadIdx.x / 16;
    if ((threadIdx.x & 15) != 0 || env >= n) return;
    for (int r = 0; r < k; r++) b[(size_t)r * n + env] = a[(size_t)r * n + env] + 1.0f;
}

static void run_soa(int n, int k) {
    float *a, *b;
    const size_t bytes = (size_t)n * k * sizeof(float);
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) { std::puts("hipMalloc"); std::exit(1); }
    hipMemset(a, 0, bytes);
    hipMemset(b, 0, bytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 10; rep++)
        hipLaunchKernelGGL(soa_kernel, dim3((unsigned)((n + 3) / 4)), dim3(64), 0, 0, a, b, n, k);
    hipDeviceSynchronize();
    std::printf("{\"kernel\": \"soa_kernel\", \"n\": %d, \"rows\": %d, \"read_bytes\": %zu, \"write_bytes\": %zu}\n", n, k,
                bytes, bytes);
    hipFree(a);
    hipFree(b);
}

template <class T>
static void run(const char* name, size_t bytes) {
    const size_t n = bytes / sizeof(T);
    T *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) { std::puts("hipMalloc"); std::exit(1); }
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 3; rep++)
        hipLaunchKernelGGL(copy_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, b, n);
    hipDeviceSynchronize();
    std::printf("{\"kernel\": \"copy_kernel<%s>\", \"read_bytes\": %zu, \"write_bytes\": %zu}\n", name, bytes, bytes);
    hipFree(a);
    hipFree(b);
}

int main() {
    const size_t bytes = (size_t)512 << 20;   // 512 MiB each way: past the 256 MiB Infinity Cache
    run<float>("float", bytes);
    run<double>("double", bytes);
    run<float4>("float4", bytes);
    run_soa(4096, 40);   // ~ the headline step kernel's rows per env (q, qd, goal, cache, counters)
    return 0;
}
