// Host cost of the HIP calls one FD batch makes, GPU box:
//   hipcc --offload-arch=gfx950 -O2 tools/api_cost.hip -o /tmp/api_cost && /tmp/api_cost
// Each line: microseconds of host time per call (the device is idle or busy
// with trivial kernels; the enqueue cost is what is measured), and for the
// graph forms the cost of a launch of a captured 4-stream, 9-kernel DAG of the
// shape enqueue_batch builds, plus the node-parameter updates a call needs.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

struct Big { char b[896]; };
__global__ void k_small(int* p, int v) { if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = v; }
__global__ void k_big(Big a, int* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = a.b[5]; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const int N = 2000;
    hipStream_t s[4];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t ev[16];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int* d = nullptr;
    CK(hipMalloc(&d, 64));
    Big big{};
    auto run = [&](const char* name, auto fn) -> int {
        for (int i = 0; i < 100; ++i) fn(i);
        CK(hipDeviceSynchronize());
        const double t0 = now_us();
        for (int i = 0; i < N; ++i) fn(i);
        const double t1 = now_us();
        CK(hipDeviceSynchronize());
        const double t2 = now_us();
        std::printf("{\"op\": \"%s\", \"issue_us\": %.2f, \"total_us\": %.2f}\n", name, (t1 - t0) / N, (t2 - t0) / N);
        return 0;
    };
    run("launch_16B_args", [&](int i) { hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, s[0], d, i); });
    run("launch_896B_args", [&](int i) { hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s[0], big, d); });
    run("launch_896B_args_dyn_lds", [&](int i) { hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 4096, s[0], big, d); });
    run("event_record", [&](int i) { (void)hipEventRecord(ev[i & 15], s[0]); });
    run("stream_wait_event", [&](int i) { (void)hipStreamWaitEvent(s[1], ev[i & 15], 0); });
    run("get_last_error", [&](int) { (void)hipGetLastError(); });
    run("set_device", [&](int) { (void)hipSetDevice(0); });
    // the FD batch pattern: 9 launches (1 + 5 + 2 + 1) on 4 streams, 4 records, 7 waits
    auto batch = [&](int i) {
        const int k = (i % 3) * 4;
        (void)hipStreamWaitEvent(s[0], ev[((i + 2) % 3) * 4 + 1], 0);
        (void)hipStreamWaitEvent(s[0], ev[((i + 2) % 3) * 4 + 3], 0);
        hipLaunchKernelGGL(k_big, dim3(544), dim3(256), 0, s[0], big, d);
        (void)hipEventRecord(ev[k + 0], s[0]);
        (void)hipStreamWaitEvent(s[1], ev[k + 0], 0);
        (void)hipStreamWaitEvent(s[1], ev[((i + 2) % 3) * 4 + 2], 0);
        for (int j = 0; j < 5; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(256), 0, s[1], big, d);
        (void)hipEventRecord(ev[k + 1], s[1]);
        (void)hipStreamWaitEvent(s[2], ev[k + 1], 0);
        (void)hipStreamWaitEvent(s[2], ev[((i + 2) % 3) * 4 + 3], 0);
        for (int j = 0; j < 2; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(64), 0, s[2], big, d);
        (void)hipEventRecord(ev[k + 2], s[2]);
        (void)hipStreamWaitEvent(s[3], ev[k + 2], 0);
        hipLaunchKernelGGL(k_big, dim3(1536), dim3(256), 0, s[3], big, d);
        (void)hipEventRecord(ev[k + 3], s[3]);
    };
    run("fd_batch_pattern_4_streams", batch);
    // the same 9 launches on one stream, no events
    run("fd_batch_pattern_1_stream", [&](int) {
        hipLaunchKernelGGL(k_big, dim3(544), dim3(256), 0, s[0], big, d);
        for (int j = 0; j < 5; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(256), 0, s[0], big, d);
        for (int j = 0; j < 2; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(64), 0, s[0], big, d);
        hipLaunchKernelGGL(k_big, dim3(1536), dim3(256), 0, s[0], big, d);
    });
    // two streams: front, and the rest (contour filter, accumulate, fix-up)
    run("fd_batch_pattern_2_streams", [&](int i) {
        const int k = (i % 3) * 2;
        (void)hipStreamWaitEvent(s[0], ev[((i + 2) % 3) * 2 + 1], 0);
        hipLaunchKernelGGL(k_big, dim3(544), dim3(256), 0, s[0], big, d);
        (void)hipEventRecord(ev[k + 0], s[0]);
        (void)hipStreamWaitEvent(s[1], ev[k + 0], 0);
        for (int j = 0; j < 8; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(256), 0, s[1], big, d);
        (void)hipEventRecord(ev[k + 1], s[1]);
    });
    // graph: capture the 4-stream DAG once, launch it N times (no updates)
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
    {
        hipLaunchKernelGGL(k_big, dim3(544), dim3(256), 0, s[0], big, d);
        CK(hipEventRecord(ev[0], s[0]));
        CK(hipStreamWaitEvent(s[1], ev[0], 0));
        for (int j = 0; j < 5; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(256), 0, s[1], big, d);
        CK(hipEventRecord(ev[1], s[1]));
        CK(hipStreamWaitEvent(s[2], ev[1], 0));
        for (int j = 0; j < 2; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(64), 0, s[2], big, d);
        CK(hipEventRecord(ev[2], s[2]));
        CK(hipStreamWaitEvent(s[3], ev[2], 0));
        hipLaunchKernelGGL(k_big, dim3(1536), dim3(256), 0, s[3], big, d);
        CK(hipEventRecord(ev[3], s[3]));
        CK(hipStreamWaitEvent(s[0], ev[3], 0));
    }
    CK(hipStreamEndCapture(s[0], &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    run("graph_launch_9_nodes", [&](int) { (void)hipGraphLaunch(ge, s[0]); });
    // graph + per-call updates of 3 kernel nodes' arguments (frame, overlay, compressed pointers)
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    CK(hipGraphGetNodes(g, nodes.data(), &nn));
    std::vector<hipGraphNode_t> kn;
    for (auto& x : nodes) {
        hipGraphNodeType t;
        CK(hipGraphNodeGetType(x, &t));
        if (t == hipGraphNodeTypeKernel) kn.push_back(x);
    }
    std::printf("{\"graph_nodes\": %zu, \"kernel_nodes\": %zu}\n", nn, kn.size());
    hipKernelNodeParams kp{};
    CK(hipGraphKernelNodeGetParams(kn[0], &kp));
    Big b2{};
    void* args[] = {&b2, &d};
    run("graph_launch_9_nodes_3_updates", [&](int i) {
        b2.b[5] = (char)i;
        hipKernelNodeParams p = kp;
        p.kernelParams = args;
        for (int j = 0; j < 3; ++j) (void)hipGraphExecKernelNodeSetParams(ge, kn[j == 0 ? 0 : kn.size() - j], &p);
        (void)hipGraphLaunch(ge, s[0]);
    });
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    // graph of the 9 kernels on ONE stream (linear chain)
    CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_big, dim3(544), dim3(256), 0, s[0], big, d);
    for (int j = 0; j < 8; ++j) hipLaunchKernelGGL(k_big, dim3(68), dim3(256), 0, s[0], big, d);
    CK(hipStreamEndCapture(s[0], &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    run("graph_launch_9_nodes_linear", [&](int) { (void)hipGraphLaunch(ge, s[0]); });
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}
