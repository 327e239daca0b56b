// Debug: which HIP runtime calls, made from the capturing thread in the relaxed capture mode, leave a
// global-mode stream capture valid? (bugseg_runtime.cpp builds BEV tables on a private stream while
// the caller's stream may be capturing.) Each case: begin capture on stream A (global mode), switch
// this thread to relaxed, make the call(s), switch back, launch a kernel on A, end capture.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/capture_probe.hip -o scripts/capture_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(int *p, int v) { p[threadIdx.x] = v; }

static const char *st(hipError_t e) { return hipGetErrorString(e); }

static void run_case(int which) {
    hipStream_t A, B = nullptr;
    (void)hipStreamCreateWithFlags(&A, hipStreamNonBlocking);
    if (which >= 10) (void)hipStreamCreateWithFlags(&B, hipStreamNonBlocking);   // B made before the capture
    int *buf = nullptr, *tmp = nullptr;
    (void)hipMalloc(&buf, 4096);
    hipError_t e = hipStreamBeginCapture(A, hipStreamCaptureModeGlobal);
    hipError_t r1 = hipSuccess, r2 = hipSuccess, r3 = hipSuccess, r4 = hipSuccess;
    {
        hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&m);
        const int w = which % 10;
        if (w >= 1 && !B) r1 = hipStreamCreateWithFlags(&B, hipStreamNonBlocking);
        if (w >= 2) r2 = hipMalloc(&tmp, 1 << 20);
        if (w >= 3) { hipLaunchKernelGGL(k_fill, dim3(1), dim3(64), 0, B, tmp, 7); r3 = hipGetLastError(); }
        if (w >= 4) r4 = hipStreamSynchronize(B);
        (void)hipThreadExchangeStreamCaptureMode(&m);
    }
    hipLaunchKernelGGL(k_fill, dim3(1), dim3(64), 0, A, buf, 1);
    hipStreamCaptureStatus cs;
    hipError_t ic = hipStreamIsCapturing(A, &cs);
    hipGraph_t g = nullptr;
    hipError_t ee = hipStreamEndCapture(A, &g);
    printf("case %2d: begin %s | create %s malloc %s launch %s sync %s | status %d (%s) | end %s\n", which, st(e), st(r1),
           st(r2), st(r3), st(r4), (int)cs, st(ic), st(ee));
    if (g) (void)hipGraphDestroy(g);
    (void)hipDeviceSynchronize();
    (void)hipGetLastError();
    if (tmp) (void)hipFree(tmp);
    (void)hipFree(buf);
    (void)hipStreamDestroy(A);
    if (B) (void)hipStreamDestroy(B);
}

int main() {
    for (int w : {0, 1, 2, 3, 4, 12, 13, 14}) run_case(w);
    return 0;
}
