// Host cost of kernel submission on this runtime: plain launches vs a captured graph.
// Prints host microseconds per launch (empty kernel, stream not synchronised in between).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(double* p, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] += 1.0;
}

__global__ void k_long(double* p, int iters)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double x = p[t];
    for (int i = 0; i < iters; i++) x = x * 0.999999 + 1e-9;
    p[t] = x;
}

static double us_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int main()
{
    double* p = nullptr;
    hipStream_t s;
    if (hipMalloc(&p, 1 << 20) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, p, 1 << 14);
    (void)hipStreamSynchronize(s);
    const int N = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, p, 1 << 14);
    const double th = us_since(t0);
    (void)hipStreamSynchronize(s);
    const double tg = us_since(t0);
    printf("plain: host %.2f us/launch, GPU drain %.2f us/launch\n", th / N, tg / N);
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 40; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, p, 1 << 14);
    (void)hipStreamEndCapture(s, &g);
    if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return 2;
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    const int G = 50;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < G; i++) (void)hipGraphLaunch(ge, s);
    const double gh = us_since(t0);
    (void)hipStreamSynchronize(s);
    const double gg = us_since(t0);
    printf("graph(40 nodes): host %.2f us/node, GPU drain %.2f us/node\n", gh / (G * 40), gg / (G * 40));
    /* fork while the main stream is busy: does the graph launch on the side stream block
     * the host until the fork point has executed? */
    hipStream_t side;
    hipEvent_t ev;
    (void)hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    for (int rep = 0; rep < 3; rep++) {
        auto t1 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_long, dim3(1), dim3(64), 0, s, p, 2000000);
        const double a = us_since(t1);
        (void)hipEventRecord(ev, s);
        (void)hipStreamWaitEvent(side, ev, 0);
        const double b = us_since(t1);
        (void)hipGraphLaunch(ge, side);
        const double c = us_since(t1);
        for (int i = 0; i < 10; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, p, 1 << 14);
        const double d = us_since(t1);
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(side);
        const double e = us_since(t1);
        printf("fork: long kernel queued %.1f us, record+wait %.1f, graph launch done %.1f, 10 more %.1f, all done %.1f\n",
               a, b, c, d, e);
    }
    /* the same with plain launches on the side stream */
    for (int rep = 0; rep < 2; rep++) {
        auto t1 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_long, dim3(1), dim3(64), 0, s, p, 2000000);
        (void)hipEventRecord(ev, s);
        (void)hipStreamWaitEvent(side, ev, 0);
        const double b = us_since(t1);
        for (int i = 0; i < 40; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, side, p, 1 << 14);
        const double c = us_since(t1);
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(side);
        printf("fork plain: record+wait %.1f, 40 side launches done %.1f, all done %.1f\n", b, c, us_since(t1));
    }
    return 0;
}
