// hipGraphLaunch host blocking probe: a linear graph of 7 spin kernels (~15 us each,
// 256 blocks) replayed back to back vs the same 7 kernels launched directly.
// Reports host us per launch call, GPU us per iteration.  Variants by argv[1]:
//   0 one exec per parity (2 execs alternating)   1 one exec only   2 + hipGraphUpload
//   3 four execs rotating   4 2 execs, launched on the NULL stream (direct launches too)
//   5 2 execs, kernels with a 2 KiB by-value argument struct
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

struct BigArgs { int* buf; long long ticks; char pad[2048]; };
__global__ void spin_big(BigArgs a) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < a.ticks) {}
    if (threadIdx.x == 0) a.buf[blockIdx.x] += 1 + a.pad[blockIdx.x & 1023];
}
__global__ void spin(int* buf, long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {}
    if (threadIdx.x == 0) buf[blockIdx.x] += 1;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int variant = argc > 1 ? atoi(argv[1]) : 0;
    int* buf;
    CK(hipMalloc(&buf, 4096 * sizeof(int)));
    CK(hipMemset(buf, 0, 4096 * sizeof(int)));
    int rate = 0;
    CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));   // kHz
    const long long ticks = (long long)rate * 15 / 1000;                    // 15 us
    hipStream_t st, cap;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
    if (variant == 4) st = nullptr;
    BigArgs ba{};
    ba.buf = buf;
    ba.ticks = ticks;
    auto launch7 = [&](hipStream_t s) {
        for (int k = 0; k < 7; ++k) {
            if (variant == 5) hipLaunchKernelGGL(spin_big, dim3(256), dim3(256), 0, s, ba);
            else hipLaunchKernelGGL(spin, dim3(256), dim3(256), 0, s, buf, ticks);
        }
    };
    const int iters = 200;
    // direct
    for (int i = 0; i < 20; ++i) launch7(st);
    CK(hipStreamSynchronize(st));
    auto t0 = std::chrono::steady_clock::now();
    double host_us = 0;
    for (int i = 0; i < iters; ++i) {
        auto a = std::chrono::steady_clock::now();
        launch7(st);
        host_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    CK(hipStreamSynchronize(st));
    double tot = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("direct: host %.1f us per 7 launches, %.1f us per iteration\n", host_us / iters, tot / iters);
    const int nexec = variant == 1 ? 1 : variant == 3 ? 4 : 2;
    std::vector<hipGraphExec_t> ex(nexec);
    for (int e = 0; e < nexec; ++e) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
        launch7(cap);
        CK(hipStreamEndCapture(cap, &g));
        CK(hipGraphInstantiate(&ex[e], g, nullptr, nullptr, 0));
        if (variant == 2) CK(hipGraphUpload(ex[e], st));
    }
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ex[i % nexec], st));
    CK(hipStreamSynchronize(st));
    t0 = std::chrono::steady_clock::now();
    host_us = 0;
    std::vector<double> each;
    for (int i = 0; i < iters; ++i) {
        auto a = std::chrono::steady_clock::now();
        CK(hipGraphLaunch(ex[i % nexec], st));
        double d = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        host_us += d;
        each.push_back(d);
    }
    CK(hipStreamSynchronize(st));
    tot = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::sort(each.begin(), each.end());
    printf("graph variant %d (%d execs): host %.1f us per hipGraphLaunch (median %.1f), %.1f us per iteration\n",
           variant, nexec, host_us / iters, each[iters / 2], tot / iters);
    return 0;
}
