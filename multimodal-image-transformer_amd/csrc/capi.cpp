// C-ABI bookkeeping for libmit_hip.so: thread-local error strings, the ABI version, and the launch
// plan recorder (mit_plan_*): a train step's ~340 launches, recorded once while the step runs for
// real and replayed from C++ afterwards, so the host pays one call per step instead of a Python
// wrapper per launch (eager semantics, multi-stream overlap intact; a hipGraph of the same step
// replays its parallel branches without overlap on ROCm 7).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include <functional>
#include <utility>
#include <vector>

#include "../../include/mit_hip.h"

static thread_local char g_err[512] = "";

int mit_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return 0;
}

extern "C" const char* mit_last_error(void) { return g_err; }
extern "C" int mit_abi_version(void) { return 6; }

// ---------------------------------------------------------------------------------------------
// launch plans
// ---------------------------------------------------------------------------------------------
struct mit_plan {
  std::vector<std::function<int()>> ops;
};

static thread_local mit_plan* g_rec = nullptr;

bool mit_plan_recording() { return g_rec != nullptr; }
void mit_plan_push(std::function<int()> op) { g_rec->ops.push_back(std::move(op)); }

extern "C" void* mit_plan_begin(void) {
  if (g_rec) {
    mit_set_error("mit_plan_begin: already recording");
    return nullptr;
  }
  g_rec = new mit_plan();
  return g_rec;
}

extern "C" void* mit_plan_end(void) {
  mit_plan* p = g_rec;
  g_rec = nullptr;
  if (!p) mit_set_error("mit_plan_end: not recording");
  return p;
}

extern "C" long mit_plan_size(const void* plan) { return plan ? (long)((const mit_plan*)plan)->ops.size() : 0; }

extern "C" int mit_plan_run(const void* plan) {
  if (!plan) {
    mit_set_error("mit_plan_run: null plan");
    return MIT_ERR_INVALID;
  }
  if (g_rec) {
    mit_set_error("mit_plan_run: cannot replay while recording");
    return MIT_ERR_INVALID;
  }
  for (const auto& op : ((const mit_plan*)plan)->ops) {
    const int rc = op();
    if (rc != MIT_OK) return rc;
  }
  return MIT_OK;
}

extern "C" void mit_plan_destroy(void* plan) { delete (mit_plan*)plan; }

// cross-stream ordering edges of a step (recordable)
extern "C" int mit_event_record(void* event, void* stream) {
  if (g_rec) g_rec->ops.push_back([=]() { return mit_event_record(event, stream); });
  const hipError_t e = hipEventRecord((hipEvent_t)event, (hipStream_t)stream);
  if (e != hipSuccess) {
    mit_set_error("mit_event_record: %s", hipGetErrorString(e));
    return MIT_ERR_HIP;
  }
  return MIT_OK;
}

extern "C" int mit_stream_wait_event(void* stream, void* event) {
  if (g_rec) g_rec->ops.push_back([=]() { return mit_stream_wait_event(stream, event); });
  const hipError_t e = hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
  if (e != hipSuccess) {
    mit_set_error("mit_stream_wait_event: %s", hipGetErrorString(e));
    return MIT_ERR_HIP;
  }
  return MIT_OK;
}
