// C ABI glue for libzonos_hip.so: error reporting, device sync and hipGraph capture of the
// decode step (the reference runs the transformer step eagerly, model.py:138-142,220-222).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>

#include <vector>

#include "../../include/zonos_hip.h"

static thread_local char g_err[1024] = "";

extern "C" void zk_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* zk_last_error(void) { return g_err; }

extern "C" int zk_version(void) { return 1; }

// sizeof / offsetof of the by-value ABI structs, so a binding (ctypes here) can verify its
// layout without a GPU: which = 0 zk_sampling_params, 1 zk_gen_state, 2 zk_small_layer,
// 3 zk_small_args, 4 ZkCondSeg, 5 ZkCondPlan; 10 + k = offset of zk_small_args' last field (prof).
extern "C" long zk_abi_size(int which) {
    switch (which) {
        case 0: return (long)sizeof(zk_sampling_params);
        case 1: return (long)sizeof(zk_gen_state);
        case 2: return (long)sizeof(zk_small_layer);
        case 3: return (long)sizeof(zk_small_args);
        case 4: return (long)sizeof(ZkCondSeg);
        case 5: return (long)sizeof(ZkCondPlan);
        case 10: return (long)offsetof(zk_small_args, prof);
        case 11: return (long)offsetof(zk_small_args, eps);
        case 12: return (long)offsetof(zk_gen_state, seed);
        default: return -1;
    }
}

extern "C" int zk_device_sync(void) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        zk_set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

#define HIPCHK(expr, what)                                                 \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e != hipSuccess) {                                            \
            zk_set_error("%s: %s", what, hipGetErrorString(_e));           \
            return -1;                                                     \
        }                                                                  \
    } while (0)

extern "C" int zk_graph_begin(void* stream) {
    HIPCHK(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal), "zk_graph_begin");
    return 0;
}

extern "C" int zk_graph_end(void* stream, void** graph_exec) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamEndCapture((hipStream_t)stream, &g), "zk_graph_end(capture)");
    hipGraphExec_t ex = nullptr;
    hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    HIPCHK(e, "zk_graph_end(instantiate)");
    *graph_exec = (void*)ex;
    return 0;
}

extern "C" int zk_graph_launch(void* graph_exec, int repeat, void* stream) {
    for (int i = 0; i < repeat; ++i)
        HIPCHK(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream), "zk_graph_launch");
    return 0;
}

extern "C" int zk_graph_destroy(void* graph_exec) {
    if (graph_exec) HIPCHK(hipGraphExecDestroy((hipGraphExec_t)graph_exec), "zk_graph_destroy");
    return 0;
}

// ---------------------------------------------------------------- event timing (bench roofline)
extern "C" int zk_event_create(void** ev) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e), "zk_event_create");
    *ev = (void*)e;
    return 0;
}
extern "C" int zk_event_record(void* ev, void* stream) {
    HIPCHK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "zk_event_record");
    return 0;
}
extern "C" int zk_event_elapsed_ms(void* a, void* b, float* ms) {
    HIPCHK(hipEventSynchronize((hipEvent_t)b), "zk_event_elapsed(sync)");
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "zk_event_elapsed");
    return 0;
}
extern "C" int zk_event_destroy(void* ev) {
    if (ev) HIPCHK(hipEventDestroy((hipEvent_t)ev), "zk_event_destroy");
    return 0;
}
