// policy.cpp — elastic-parallelism scheduling policies (native control-plane core).
//
// Re-implements the reference's ThroughputBasedPolicy (ml/pkg/scheduler/policy.go:50-102)
// as a thread-safe native component, fixing the two reference defects called out in
// the decision is clamped to [min_p, max_p] (the reference could
// reach 0 or go negative) and every cache access is under the lock (the reference
// wrote its timeCache through value receivers without the lock).
//
// Decision rule per job (elapsed = last epoch's wall time):
//   first sight                          -> default parallelism, op CREATE
//   cached reference time == 0           -> p + 1, reference := elapsed
//   elapsed <= ref * scale_up (1.05)     -> p + 1, reference := elapsed
//   elapsed >= ref * scale_down (1.2)    -> p - 1, reference := elapsed
//   otherwise                            -> p (reference kept)
#include <mutex>
#include <string>
#include <unordered_map>

#define KML_API extern "C" __attribute__((visibility("default")))

namespace {

struct Policy {
  double scale_up = 1.05, scale_down = 1.2;
  int min_p = 1, max_p = 8;
  std::mutex mu;
  std::unordered_map<std::string, double> time_cache;
};

int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace

KML_API void* kml_policy_new(double scale_up, double scale_down, int min_p, int max_p) {
  Policy* p = new Policy();
  p->scale_up = scale_up;
  p->scale_down = scale_down;
  p->min_p = min_p < 1 ? 1 : min_p;
  p->max_p = max_p < p->min_p ? p->min_p : max_p;
  return p;
}

KML_API void kml_policy_free(void* h) { delete static_cast<Policy*>(h); }

KML_API void kml_policy_set_bounds(void* h, int min_p, int max_p) {
  Policy* p = static_cast<Policy*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  p->min_p = min_p < 1 ? 1 : min_p;
  p->max_p = max_p < p->min_p ? p->min_p : max_p;
}

// op_out: 0 = CREATE_TASK, 1 = UPDATE_TASK
KML_API int kml_policy_decide(void* h, const char* job_id, int default_parallelism, int parallelism,
                              double elapsed, int* op_out) {
  Policy* p = static_cast<Policy*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  const std::string id(job_id);
  auto it = p->time_cache.find(id);
  if (it == p->time_cache.end()) {
    p->time_cache[id] = 0.0;
    *op_out = 0;
    return clampi(default_parallelism, p->min_p, p->max_p);
  }
  *op_out = 1;
  const double prev = it->second;
  int next;
  if (prev == 0.0) {
    it->second = elapsed;
    next = parallelism + 1;
  } else if (elapsed <= prev * p->scale_up) {
    it->second = elapsed;
    next = parallelism + 1;
  } else if (elapsed >= prev * p->scale_down) {
    it->second = elapsed;
    next = parallelism - 1;
  } else {
    next = parallelism;
  }
  return clampi(next, p->min_p, p->max_p);
}

KML_API void kml_policy_finish(void* h, const char* job_id) {
  Policy* p = static_cast<Policy*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  p->time_cache.erase(std::string(job_id));
}

KML_API double kml_policy_reference_time(void* h, const char* job_id) {
  Policy* p = static_cast<Policy*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->time_cache.find(std::string(job_id));
  return it == p->time_cache.end() ? -1.0 : it->second;
}
