// Error reporting and conv launch timing for liboflow.
#include "common.h"

#include <mutex>
#include <unordered_map>
#include <vector>

namespace oflow {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(OF_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  return OF_OK;
}

int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;
  }
  int v = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (v > 0) return v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      v <= 0) {
    (void)hipGetLastError();
    v = 256;
  }
  __atomic_store_n(&cache[dev], v, __ATOMIC_RELAXED);
  return v;
}

// ---- timing: hipEvent pairs recorded on the launch stream, read back on demand ----------
struct TimedLaunch {
  int kind;
  double flops;
  hipEvent_t start, stop;
};

static std::mutex g_tmu;
static bool g_timing = false;
static bool g_timing_oneshot = false;   // of_timing_enable(2): the next conv launch only
static std::vector<TimedLaunch> g_launches;
static std::vector<hipEvent_t> g_event_pool;
static hipEvent_t g_pending_start = nullptr;

static hipEvent_t get_event() {
  if (!g_event_pool.empty()) {
    hipEvent_t e = g_event_pool.back();
    g_event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

bool timing_on() { return g_timing; }

// Inside a stream capture (HIP graph) a plain hipEventRecord only expresses a dependency;
// hipEventRecordExternal makes it an event-record node, so every replay of the graph
// re-records the pair and of_timing_read() returns the durations of the latest replay.
static void record(hipEvent_t e, hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive) {
    if (hipEventRecordWithFlags(e, s, hipEventRecordExternal) != hipSuccess)
      (void)hipGetLastError();   // not recorded: leave no sticky error for the next launch check
  } else {
    (void)hipEventRecord(e, s);
  }
}

void timing_begin(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_pending_start = get_event();
  if (g_pending_start) record(g_pending_start, s);
}

void timing_end(hipStream_t s, int kind, double flops) {
  std::lock_guard<std::mutex> lk(g_tmu);
  if (!g_pending_start) return;
  hipEvent_t stop = get_event();
  if (!stop) return;
  record(stop, s);
  g_launches.push_back({kind, flops, g_pending_start, stop});
  g_pending_start = nullptr;
  if (g_timing_oneshot) g_timing = g_timing_oneshot = false;
}

// ---- cross-stream ordering --------------------------------------------------------------
// A default hipEvent releases at system scope when it is recorded and its waiters acquire at
// system scope; ordering two streams of one device needs device scope only.  A ring of
// fence-light events per device (hipStreamWaitEvent binds the record current at the call,
// so re-recording a ring slot later is safe).
static std::mutex g_wmu;
struct WaitRing {
  std::vector<hipEvent_t> ev;
  size_t next = 0;
};
static std::unordered_map<int, WaitRing> g_wait_rings;
constexpr int kWaitRing = 64;

}  // namespace oflow

using namespace oflow;

extern "C" {

int of_abi_version(void) { return OF_ABI_VERSION; }

const char* of_last_error(void) { return g_last_error.c_str(); }

int of_same_pads(int n, int k, int s, int* before, int* after, int* out) {
  OF_CHECK_ARG(n > 0 && k > 0 && s > 0 && before && after && out, "same_pads: args");
  const int o = (n + s - 1) / s;
  int total = (o - 1) * s + k - n;
  if (total < 0) total = 0;
  *before = total / 2;
  *after = total - total / 2;
  *out = o;
  return OF_OK;
}

int of_stream_wait(void* waiter, void* signaller) {
  OF_CHECK_ARG(waiter != signaller, "stream_wait: waiter and signaller are one stream");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return check_launch("stream_wait: hipGetDevice");
  hipEvent_t e = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_wmu);
    WaitRing& r = g_wait_rings[dev];
    if (r.ev.empty()) {
      for (int i = 0; i < kWaitRing; ++i) {
        hipEvent_t x = nullptr;
        if (hipEventCreateWithFlags(&x, hipEventDisableTiming | hipEventDisableSystemFence) !=
            hipSuccess)
          return check_launch("stream_wait: hipEventCreateWithFlags");
        r.ev.push_back(x);
      }
    }
    e = r.ev[r.next++ % r.ev.size()];
  }
  if (hipEventRecord(e, static_cast<hipStream_t>(signaller)) != hipSuccess)
    return check_launch("stream_wait: hipEventRecord");
  if (hipStreamWaitEvent(static_cast<hipStream_t>(waiter), e, 0) != hipSuccess)
    return check_launch("stream_wait: hipStreamWaitEvent");
  return OF_OK;
}

int of_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_tmu);
  OF_CHECK_ARG(on >= 0 && on <= 2, "timing_enable: 0, 1 or 2");
  g_timing = on != 0;
  g_timing_oneshot = on == 2;
  return OF_OK;
}

int of_timing_read(int max, int* kinds, double* flops, float* ms) {
  std::lock_guard<std::mutex> lk(g_tmu);
  int n = 0;
  for (auto& t : g_launches) {
    if (hipEventSynchronize(t.stop) != hipSuccess) return -1;
    if (n < max) {
      float e = 0.f;
      (void)hipEventElapsedTime(&e, t.start, t.stop);
      if (kinds) kinds[n] = t.kind;
      if (flops) flops[n] = t.flops;
      if (ms) ms[n] = e;
    }
    ++n;
    g_event_pool.push_back(t.start);
    g_event_pool.push_back(t.stop);
  }
  g_launches.clear();
  return n < max ? n : max;
}

}  // extern "C"
