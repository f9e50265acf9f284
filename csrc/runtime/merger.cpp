// merger.cpp — host-side model merger (the reference's hot path, re-done natively).
//
// The reference TrainJob sums every function's weights into the reference model on
// one CPU under a mutex and then divides by n (ml/pkg/model/model.go:249-302,
// ml/pkg/model/parallelSGD.go:26-54).  On MI355X the averaging of GPU workers is an
// RCCL all-reduce; this merger serves the CPU workers of the plumbing config and the
// in-process ThreadComm backend: a multi-threaded, vectorisable sum / average over N
// equally sized fp32 buffers, summed in rank order (deterministic).
#include <algorithm>
#include <cstddef>
#include <thread>
#include <vector>

#define KML_API extern "C" __attribute__((visibility("default")))

namespace {

void sum_range(float* out, const float* const* srcs, int n, size_t b, size_t e, float scale) {
  for (size_t i = b; i < e; ++i) {
    float acc = 0.f;
    for (int r = 0; r < n; ++r) acc += srcs[r][i];
    out[i] = acc * scale;
  }
}

int run(float* out, const float* const* srcs, int n, long long numel, int threads, float scale) {
  if (n <= 0 || numel < 0) return 1;
  const size_t N = (size_t)numel;
  threads = std::max(1, std::min(threads, 64));
  if (threads == 1 || N < (1u << 16)) {
    sum_range(out, srcs, n, 0, N, scale);
    return 0;
  }
  std::vector<std::thread> ts;
  const size_t per = (N + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t b = t * per, e = std::min(N, b + per);
    if (b >= e) break;
    ts.emplace_back(sum_range, out, srcs, n, b, e, scale);
  }
  for (auto& t : ts) t.join();
  return 0;
}

}  // namespace

// out = sum_r srcs[r]
KML_API int kml_sum_f32(float* out, const float* const* srcs, int n, long long numel, int threads) {
  return run(out, srcs, n, numel, threads, 1.f);
}

// out = (1/n) sum_r srcs[r]
KML_API int kml_average_f32(float* out, const float* const* srcs, int n, long long numel, int threads) {
  return run(out, srcs, n, numel, threads, n > 0 ? 1.f / (float)n : 0.f);
}

// dst += src (reference Model.Update accumulate step)
KML_API int kml_accumulate_f32(float* dst, const float* src, long long numel) {
  for (long long i = 0; i < numel; ++i) dst[i] += src[i];
  return 0;
}
