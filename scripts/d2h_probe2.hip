// Which engine carries a 402 MB device -> page-locked host copy when it follows kernels, as inside the
// engine (one act: a chain's kernels, then its observations leave): run under rocprofv3 --kernel-trace
// --memory-copy-trace (a blit shows as __amd_rocclr_copyBuffer, an SDMA copy as a memory copy).
//   A: stream i of 4 (created like the engine's): busy kernel, then the copy on the same stream
//   B: the copy on its own stream after a hipStreamWaitEvent on stream i's kernel
//   C: the copy on stream i with nothing before it
//   D: two copies in flight on two streams at once, each after its own kernel
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void busy(float *out, long long ticks) {
    const long long t0 = wall_clock64();
    float a = threadIdx.x;
    while (wall_clock64() - t0 < ticks) a = a * 1.0001f + 0.5f;
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

static double since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    const size_t n = (size_t)32768 * 12288;
    void *d = nullptr, *h = nullptr, *h2 = nullptr;
    float *scratch = nullptr;
    CK(hipMalloc(&d, 2 * n));
    CK(hipMemset(d, 1, 2 * n));
    CK(hipMalloc(&scratch, 1024 * 64 * sizeof(float)));
    h = aligned_alloc(4096, n);
    h2 = aligned_alloc(4096, n);
    CK(hipHostRegister(h, n, hipHostRegisterDefault));
    CK(hipHostRegister(h2, n, hipHostRegisterDefault));
    hipStream_t s[5];
    for (int i = 0; i < 5; i++) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const long long ticks = 100000; // 1 ms at the 100 MHz wall clock
    for (int i = 0; i < 4; i++) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s[i], scratch, ticks);
        CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s[i]));
        CK(hipStreamSynchronize(s[i]));
        printf("A stream %d: kernel + copy %.2f ms\n", i, since(t0) * 1e3);
    }
    for (int i = 0; i < 4; i++) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s[i], scratch, ticks);
        CK(hipEventRecord(ev, s[i]));
        CK(hipStreamWaitEvent(s[4], ev, 0));
        CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s[4]));
        CK(hipStreamSynchronize(s[4]));
        printf("B copy stream after stream %d: %.2f ms\n", i, since(t0) * 1e3);
    }
    for (int i = 0; i < 4; i++) {
        auto t0 = std::chrono::steady_clock::now();
        CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s[i]));
        CK(hipStreamSynchronize(s[i]));
        printf("C stream %d: copy alone %.2f ms\n", i, since(t0) * 1e3);
    }
    {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s[0], scratch, ticks);
        hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s[1], scratch, ticks);
        CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s[0]));
        CK(hipMemcpyAsync(h2, (uint8_t *)d + n, n, hipMemcpyDeviceToHost, s[1]));
        CK(hipDeviceSynchronize());
        printf("D two copies on streams 0, 1: %.2f ms\n", since(t0) * 1e3);
    }
    CK(hipHostUnregister(h));
    CK(hipHostUnregister(h2));
    free(h);
    free(h2);
    return 0;
}
