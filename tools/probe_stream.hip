// probe_stream.hip — the HIP runtime's first-queue cost, apart from this library: device count,
// one malloc, then (mode 0) hipStreamCreateWithFlags + a launch on it, or (mode 1) the first launch
// on the null stream; then a second stream and a launch on it.  One JSON line, wall-clock ms.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe_stream.hip -o build/probe_stream
// (profiles/probe_stream_r05i.jsonl)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
__global__ void k(int* p) { if (p) p[threadIdx.x] = threadIdx.x; }
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
    int mode = atoi(argv[1]);
    double t0 = ms(); int n = 0; (void)hipGetDeviceCount(&n); double t1 = ms();
    int* d = nullptr; (void)hipMalloc(&d, 4096); double t2 = ms();
    hipStream_t s = nullptr;
    if (mode == 0) { (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }
    double t3 = ms();
    k<<<1, 64, 0, s>>>(d); (void)hipStreamSynchronize(s); double t4 = ms();
    hipStream_t s2 = nullptr; (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking); double t5 = ms();
    k<<<1, 64, 0, s2>>>(d); (void)hipStreamSynchronize(s2); double t6 = ms();
    printf("{\"mode\": %d, \"devcount\": %.2f, \"malloc\": %.2f, \"stream_create\": %.2f, \"first_launch_sync\": %.2f, \"second_stream_create\": %.2f, \"second_launch\": %.2f}\n", mode, t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5);
    return 0;
}
