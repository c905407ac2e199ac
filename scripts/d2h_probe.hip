// Which engine carries a device -> host copy into (a) hipHostMalloc'd and (b) malloc'd +
// hipHostRegister'd memory, on a non-blocking stream: run under rocprofv3 --kernel-trace
// --memory-copy-trace (a blit shows as __amd_rocclr_copyBuffer, an SDMA copy as a memory copy).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static double run(void *dst, const void *src, size_t n, hipStream_t s) {
    double best = 0;
    for (int i = 0; i < 3; i++) {
        auto t0 = std::chrono::steady_clock::now();
        if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
        if (hipStreamSynchronize(s) != hipSuccess) return -1;
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = best > n / dt ? best : n / dt;
    }
    return best / 1e9;
}

int main() {
    const size_t n = (size_t)32768 * 12288;
    void *d = nullptr, *h1 = nullptr;
    CK(hipMalloc(&d, n));
    CK(hipMemset(d, 1, n));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipHostMalloc(&h1, n, hipHostMallocDefault));
    printf("hipHostMalloc     : %.1f GB/s\n", run(h1, d, n, s));
    void *h2 = aligned_alloc(4096, n);
    CK(hipHostRegister(h2, n, hipHostRegisterDefault));
    printf("hipHostRegister   : %.1f GB/s\n", run(h2, d, n, s));
    CK(hipHostUnregister(h2));
    free(h2);
    CK(hipHostFree(h1));
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
    return 0;
}
