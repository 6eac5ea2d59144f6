// capture_mode_probe.hip -- what HIP returns to a SECOND host thread that queries an event while
// the first thread is capturing a stream into a graph, for each hipStreamCaptureMode.
//
// This is the situation of torch's ProcessGroupNCCL watchdog thread (it polls the end events of
// eager collectives with hipEventQuery) while bench.py / tests capture a step with
// torch.cuda.graph(...) (default mode: global).  Nothing here can fault the GPU: two trivial
// kernels, one completed event, queries and a graph launch.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -pthread tools/capture_mode_probe.hip -o tools/capture_mode_probe
//   tools/capture_mode_probe global|thread_local|relaxed      (one mode per process: a global-mode
//   capture that another thread invalidates leaves the capturing stream unusable afterwards)
#include <hip/hip_runtime.h>

#include <atomic>
#include <string>
#include <cstdio>
#include <thread>

__global__ void bump(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

static const char* mode_name(hipStreamCaptureMode m) {
    return m == hipStreamCaptureModeGlobal ? "global" : m == hipStreamCaptureModeThreadLocal ? "thread_local"
                                                                                            : "relaxed";
}

int main(int argc, char** argv) {
    const std::string want = argc > 1 ? argv[1] : "global";
    int* d = nullptr;
    if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 1;
    (void)hipMemset(d, 0, sizeof(int));
    hipStream_t cap, other;
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&other, hipStreamNonBlocking);
    hipEvent_t done;
    (void)hipEventCreateWithFlags(&done, hipEventDisableTiming);
    bump<<<1, 64, 0, other>>>(d);
    (void)hipEventRecord(done, other);
    (void)hipDeviceSynchronize();

    const hipStreamCaptureMode modes[3] = {hipStreamCaptureModeGlobal, hipStreamCaptureModeThreadLocal,
                                           hipStreamCaptureModeRelaxed};
    int bad = 0;
    for (hipStreamCaptureMode m : modes) {
        if (want != mode_name(m)) continue;
        std::atomic<int> stage{0};
        hipError_t q_event = hipSuccess, q_stream = hipSuccess, q_last = hipSuccess;
        std::thread watchdog([&] {
            while (stage.load() != 1) std::this_thread::yield();
            q_event = hipEventQuery(done);          // what ProcessGroupNCCL's watchdog calls
            q_stream = hipStreamQuery(other);
            q_last = hipGetLastError();
            stage.store(2);
        });
        hipError_t b = hipStreamBeginCapture(cap, m);
        bump<<<1, 64, 0, cap>>>(d);
        stage.store(1);
        while (stage.load() != 2) std::this_thread::yield();
        bump<<<1, 64, 0, cap>>>(d);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(cap, &g);
        watchdog.join();
        hipGraphExec_t ge = nullptr;
        hipError_t inst = g ? hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) : hipErrorInvalidValue;
        hipError_t launch = ge ? hipGraphLaunch(ge, cap) : hipErrorInvalidValue;
        hipError_t sync = hipStreamSynchronize(cap);
        (void)hipGetLastError();
        printf("{\"mode\": \"%s\", \"begin\": \"%s\", \"other_thread_event_query\": \"%s\", "
               "\"other_thread_stream_query\": \"%s\", \"other_thread_last_error\": \"%s\", \"end_capture\": \"%s\", "
               "\"instantiate\": \"%s\", \"replay\": \"%s\", \"sync\": \"%s\"}\n",
               mode_name(m), hipGetErrorName(b), hipGetErrorName(q_event), hipGetErrorName(q_stream),
               hipGetErrorName(q_last), hipGetErrorName(e), hipGetErrorName(inst), hipGetErrorName(launch),
               hipGetErrorName(sync));
        if (ge) (void)hipGraphExecDestroy(ge);
        if (g) (void)hipGraphDestroy(g);
        if (sync != hipSuccess) bad = 1;
    }
    (void)hipDeviceSynchronize();
    (void)hipFree(d);
    (void)bad;
    return 0;   // a report, not a check: the JSON line says what HIP returned
}
