// Launch plans: record a sequence of the library's launches once, re-issue it from C++.
//
// The step engine (cgan3d_amd/engine.py) issues ~200 launches per G+D step through the ctypes
// wrappers; their host cost (~10 us each: operand checks, argument marshalling) exceeded the GPU
// time of the step.  A plan records what the entry points would enqueue — kernel launches with
// their by-value arguments, workspace memsets, cross-stream waits — and cgan3d_plan_run re-issues
// them in order on the recorded streams, so the whole step costs one ctypes call plus one
// hipLaunchKernel per kernel.  Unlike a replayed hipGraph the two-stream structure (weight
// gradients beside the input-gradient chain) is kept exactly as in eager mode.
//
// Contract (as for hipGraph capture): every buffer and device scalar a recorded launch touches
// must stay allocated and keep its address; values may change between runs.
#include <cstring>
#include <string>

#include "common.h"

namespace cg {

thread_local Plan* g_rec = nullptr;

static hipEvent_t g_eager_events[64];
static int g_eager_next = -1;

// Cross-stream waits join two streams of one device, so the event's release only has to reach
// device scope: hipEventDisableSystemFence skips the system-scope cache write-back a default event
// record issues (CGAN3D_DEBUG=system_fence restores it for A/B runs).
static unsigned event_flags() {
  static const unsigned f = [] {
    const char* v = getenv("CGAN3D_DEBUG");
    const bool sys = v && strstr(v, "system_fence") != nullptr;
    return hipEventDisableTiming | (sys ? 0u : (unsigned)hipEventDisableSystemFence);
  }();
  return f;
}

// CGAN3D_DEBUG=event_record: every cross-stream wait records its own marker event (A/B runs).
static bool bind_disabled() {
  static const bool off = [] {
    const char* v = getenv("CGAN3D_DEBUG");
    return v && strstr(v, "event_record") != nullptr;
  }();
  return off;
}

static thread_local std::string g_time_filter;  // cgan3d_plan_time_filter

bool plan_time_match(const void* k, hipStream_t st) {  // the filter: substrings separated by '|'
  if (g_time_filter.empty()) return false;
  const char* n = hipKernelNameRefByPtr(k, st);
  if (n == nullptr) return false;
  size_t b = 0;
  while (b <= g_time_filter.size()) {
    size_t e = g_time_filter.find('|', b);
    if (e == std::string::npos) e = g_time_filter.size();
    if (e > b && strstr(n, g_time_filter.substr(b, e - b).c_str()) != nullptr) return true;
    b = e + 1;
  }
  return false;
}

}  // namespace cg

using namespace cg;

extern "C" int cgan3d_plan_time_filter(const char* substring) {
  g_time_filter = substring ? substring : "";
  return CGAN3D_OK;
}

extern "C" int64_t cgan3d_plan_times(void* plan, float* ms, int64_t max) {
  if (plan == nullptr) return -1;
  Plan* p = static_cast<Plan*>(plan);
  const int64_t n = (int64_t)p->timed.size();
  for (int64_t i = 0; i < n && i < max && ms != nullptr; ++i) {
    float v = -1.f;
    if (hipEventElapsedTime(&v, p->timed[i].first, p->timed[i].second) != hipSuccess) v = -1.f;
    ms[i] = v;
  }
  return n;
}

extern "C" int cgan3d_plan_begin(void) {
  CG_CHECK_ARG(g_rec == nullptr, "cgan3d_plan_begin: a plan is already being recorded on this thread");
  g_rec = new Plan();
  return CGAN3D_OK;
}

extern "C" int cgan3d_plan_end(void** plan) {
  CG_CHECK_ARG(g_rec != nullptr, "cgan3d_plan_end: no plan is being recorded");
  CG_CHECK_ARG(plan != nullptr, "cgan3d_plan_end: null output");
  *plan = g_rec;
  g_rec = nullptr;
  return CGAN3D_OK;
}

extern "C" int64_t cgan3d_plan_size(void* plan) {
  return plan ? (int64_t)static_cast<Plan*>(plan)->ops.size() : 0;
}

extern "C" int cgan3d_plan_run(void* plan) {
  CG_CHECK_ARG(plan != nullptr, "cgan3d_plan_run: null plan");
  CG_CHECK_ARG(g_rec == nullptr, "cgan3d_plan_run: cannot run a plan while recording");
  Plan* p = static_cast<Plan*>(plan);
  for (size_t i = 0; i < p->ops.size(); ++i) {
    const hipError_t e = p->ops[i]();
    if (e != hipSuccess) {
      set_error("cgan3d_plan_run: op %zu of %zu failed: %s", i, p->ops.size(), hipGetErrorString(e));
      return CGAN3D_EHIP;
    }
  }
  return CGAN3D_OK;
}

extern "C" int cgan3d_plan_destroy(void* plan) {
  if (plan == nullptr) return CGAN3D_OK;
  Plan* p = static_cast<Plan*>(plan);
  for (hipEvent_t e : p->events) (void)hipEventDestroy(e);
  delete p;
  return CGAN3D_OK;
}

// `waiter` waits for everything enqueued so far on `signaler` (torch's Stream.wait_stream).
extern "C" int cgan3d_stream_wait(void* waiter, void* signaler) {
  hipStream_t w = static_cast<hipStream_t>(waiter), s = static_cast<hipStream_t>(signaler);
  if (w == s) return CGAN3D_OK;
  hipEvent_t ev;
  if (g_rec != nullptr) {
    // Bind to the signaler's last launch when there is one: the waiter then depends on that
    // dispatch's completion signal, and the signaler's queue carries no extra barrier packet (a
    // hipEventRecord marker costs the signaling stream ~5 us of dispatch bubble on this pool; see
    // DESIGN.md §5).  Anything else last on the signaler (a memset, a collective, a wait — whose
    // dependencies must carry over transitively) keeps the recorded marker.
    auto it = g_rec->tail.find(s);
    std::shared_ptr<hipEvent_t> slot = (it != g_rec->tail.end() && !bind_disabled()) ? it->second : nullptr;
    if (slot && *slot != nullptr) {
      ev = *slot;
    } else {
      if (hipEventCreateWithFlags(&ev, event_flags()) != hipSuccess) {
        set_error("cgan3d_stream_wait: hipEventCreate failed");
        return CGAN3D_EHIP;
      }
      g_rec->events.push_back(ev);
      if (slot) *slot = ev;
    }
    if (slot)
      g_rec->add([ev, w]() { return hipStreamWaitEvent(w, ev, 0); }, w);
    else
      g_rec->add([ev, w, s]() {
        hipError_t e = hipEventRecord(ev, s);
        return e != hipSuccess ? e : hipStreamWaitEvent(w, ev, 0);
      }, w);
    return CGAN3D_OK;
  }
  // eager: a small ring (an event may be re-recorded once the wait on it has been enqueued)
  if (g_eager_next < 0) {
    for (auto& e : g_eager_events)
      if (hipEventCreateWithFlags(&e, event_flags()) != hipSuccess) {
        set_error("cgan3d_stream_wait: hipEventCreate failed");
        return CGAN3D_EHIP;
      }
    g_eager_next = 0;
  }
  ev = g_eager_events[g_eager_next];
  g_eager_next = (g_eager_next + 1) % 64;
  if (hipEventRecord(ev, s) != hipSuccess || hipStreamWaitEvent(w, ev, 0) != hipSuccess) {
    set_error("cgan3d_stream_wait: event record/wait failed");
    return CGAN3D_EHIP;
  }
  return CGAN3D_OK;
}

// the timed launches of the last run as a timeline: start / end (ms) relative to the first timed launch's
// start, the stream (index in order of first appearance among the timed launches); returns the count
extern "C" int64_t cgan3d_plan_timeline(void* plan, float* start_ms, float* end_ms, int32_t* stream_id, int64_t max) {
  if (plan == nullptr) return -1;
  Plan* p = static_cast<Plan*>(plan);
  const int64_t n = (int64_t)p->timed.size();
  std::vector<hipStream_t> seen;
  for (int64_t i = 0; i < n && i < max; ++i) {
    float a = -1.f, b = -1.f;
    if (hipEventElapsedTime(&a, p->timed[0].first, p->timed[i].first) != hipSuccess) a = -1.f;
    if (hipEventElapsedTime(&b, p->timed[0].first, p->timed[i].second) != hipSuccess) b = -1.f;
    if (start_ms) start_ms[i] = a;
    if (end_ms) end_ms[i] = b;
    int sid = -1;
    for (size_t k = 0; k < seen.size(); ++k)
      if (seen[k] == p->timed_what[i].first) sid = (int)k;
    if (sid < 0) { sid = (int)seen.size(); seen.push_back(p->timed_what[i].first); }
    if (stream_id) stream_id[i] = sid;
  }
  return n;
}

// the (mangled) kernel name of timed launch i, or NULL
extern "C" const char* cgan3d_plan_timed_name(void* plan, int64_t i) {
  Plan* p = static_cast<Plan*>(plan);
  if (p == nullptr || i < 0 || i >= (int64_t)p->timed_what.size()) return nullptr;
  return hipKernelNameRefByPtr(p->timed_what[i].second, p->timed_what[i].first);
}
