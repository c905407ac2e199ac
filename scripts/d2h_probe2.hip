// Which engine carries a 402 MB device -> page-locked host copy when it follows kernels, as inside the
// engine (one act: a chain's kernels, then its observations leave): run under rocprofv3 --kernel-trace
// --memory-copy-trace (a blit shows as __amd_rocclr_copyBuffer, an SDMA copy as a memory copy).
//   A: stream i of 4 (created like the engine's): busy kernel, then the copy on the same stream
//   B: the copy on its own stream after a hipStreamWaitEvent on stream i's kernel
//   C: the copy on stream i with nothing before it
//   D: two copies in flight on two streams at once, each after its own kernel
// Built as an executable (main) and as a library (d2h_probe2.so, d2h_probe()) that
// scripts/d2h_probe_torch.py calls inside a Python process with and without torch's HIP context.
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

extern "C" int d2h_probe(void) {
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
    // release everything before returning to the caller: the round-5 Python run under rocprofv3 left the
    // streams, the event and both device buffers to the runtime's static teardown, and a destructor then ran
    // after the HIP / profiler libraries were gone (SIGSEGV in __cxa_finalize, gpurun_out/n/torch.log)
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 5; i++) CK(hipStreamDestroy(s[i]));
    CK(hipEventDestroy(ev));
    CK(hipHostUnregister(h));
    CK(hipHostUnregister(h2));
    free(h);
    free(h2);
    CK(hipFree(d));
    CK(hipFree(scratch));
    return 0;
}

// E: the copy after a kernel into a caller-supplied buffer (a numpy array from Python), registered here
extern "C" int d2h_probe_host(void *h) {
    const size_t n = (size_t)32768 * 12288;
    void *d = nullptr;
    float *scratch = nullptr;
    CK(hipMalloc(&d, n));
    CK(hipMalloc(&scratch, 1024 * 64 * sizeof(float)));
    CK(hipHostRegister(h, n, hipHostRegisterDefault));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s, scratch, 100000LL);
        CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("E caller buffer %p: kernel + copy %.2f ms\n", h, since(t0) * 1e3);
    }
    CK(hipStreamSynchronize(s));
    CK(hipHostUnregister(h));
    CK(hipStreamDestroy(s));
    CK(hipFree(d));
    CK(hipFree(scratch));
    return 0;
}

// F-I: the engine's conditions one at a time, each timed (SDMA 7.06 ms, blit ~7.4 ms per 402 MB):
//   F priority streams exist in the process, G the source inside a 3.3 GB allocation (at offset 2.9 GB),
//   H the destination at an offset inside a larger registered region, I hipMemcpyDefault / DtoH API
extern "C" int d2h_probe_engine_like(void) {
    const size_t n = (size_t)32768 * 12288;
    float *scratch = nullptr;
    CK(hipMalloc(&scratch, 1024 * 64 * sizeof(float)));
    auto timed = [&](const char *what, void *dst, const void *src, hipStream_t s, int api) -> int {
        for (int i = 0; i < 2; i++) {
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(busy, dim3(1024), dim3(64), 0, s, scratch, 100000LL);
            hipError_t e = api == 0   ? hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s)
                           : api == 1 ? hipMemcpyAsync(dst, src, n, hipMemcpyDefault, s)
                                      : hipMemcpyDtoHAsync(dst, (hipDeviceptr_t)src, n, s);
            if (e != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return 1;
            printf("%s: kernel + copy %.2f ms\n", what, since(t0) * 1e3);
        }
        return 0;
    };
    void *d = nullptr, *big = nullptr;
    CK(hipMalloc(&d, n));
    void *h = aligned_alloc(4096, 3 * n);
    CK(hipHostRegister(h, 3 * n, hipHostRegisterDefault));
    hipStream_t s, ph, pl;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (timed("base", h, d, s, 0)) return 1;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&ph, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&pl, hipStreamNonBlocking, lo));
    if (timed("F priority streams exist", h, d, s, 0)) return 1;
    if (timed("F copy on the high-priority stream", h, d, ph, 0)) return 1;
    CK(hipMalloc(&big, 8 * n + 4096));
    if (timed("G source at 2.9 GB in a 3.3 GB allocation", h, (uint8_t *)big + 7 * n, s, 0)) return 1;
    if (timed("H destination at +402 MB in a 1.2 GB registered region", (uint8_t *)h + n, d, s, 0)) return 1;
    if (timed("H destination at +16 B", (uint8_t *)h + 16, d, s, 0)) return 1;
    if (timed("I hipMemcpyDefault", h, d, s, 1)) return 1;
    if (timed("I hipMemcpyDtoHAsync", h, d, s, 2)) return 1;
    CK(hipDeviceSynchronize());
    CK(hipStreamDestroy(s));
    CK(hipStreamDestroy(ph));
    CK(hipStreamDestroy(pl));
    CK(hipHostUnregister(h));
    free(h);
    CK(hipFree(d));
    CK(hipFree(big));
    CK(hipFree(scratch));
    return 0;
}

#ifndef D2H_PROBE_LIB
int main() { return d2h_probe() || d2h_probe_engine_like(); }
#endif
