// Host-only tests of the native runtime (policy, merger, npy loader), built twice by
// tests/test_sanitize_cpu.py — AddressSanitizer + UndefinedBehaviorSanitizer, and
// ThreadSanitizer — and run without a GPU (sanitizers on the C++ runtime's host
// code; GPU ASan is not available).  Hammers the policy from several threads (the reference's
// policy had unlocked map writes, policy.go:70-84) and drives the loader's fill thread with
// concurrent push / take / pending calls from three threads.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* kml_policy_new(double, double, int, int);
void kml_policy_free(void*);
void kml_policy_set_bounds(void*, int, int);
int kml_policy_decide(void*, const char*, int, int, double, int*);
void kml_policy_finish(void*, const char*);
double kml_policy_reference_time(void*, const char*);
int kml_sum_f32(float*, const float* const*, int, long long, int);
int kml_average_f32(float*, const float* const*, int, long long, int);
int kml_accumulate_f32(float*, const float*, long long);
void* kml_npy_open(const char*);
void kml_npy_close(void*);
int kml_npy_info(void*, long long*);
int kml_npy_gather(void*, long long, long long, void*, int);
void* kml_prefetch_new(void*, int, long long);
long long kml_prefetch_push(void*, long long, long long);
long long kml_prefetch_take_host(void*, void*);
long long kml_prefetch_pending(void*);
void kml_prefetch_free(void*);
}

static int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static void test_policy() {
  void* p = kml_policy_new(1.05, 1.2, 1, 8);
  int op = -1;
  CHECK(kml_policy_decide(p, "j", 2, 0, 0.0, &op) == 2 && op == 0);   // create
  CHECK(kml_policy_decide(p, "j", 2, 2, 10.0, &op) == 3 && op == 1);  // no reference yet -> +1
  CHECK(kml_policy_decide(p, "j", 2, 3, 10.4, &op) == 4);             // <= 1.05x -> +1
  CHECK(kml_policy_decide(p, "j", 2, 4, 11.5, &op) == 4);             // between -> keep
  CHECK(kml_policy_decide(p, "j", 2, 4, 13.0, &op) == 3);             // >= 1.2x -> -1
  kml_policy_finish(p, "j");
  CHECK(kml_policy_decide(p, "j", 5, 0, 0.0, &op) == 5 && op == 0);
  // clamp
  kml_policy_set_bounds(p, 1, 2);
  CHECK(kml_policy_decide(p, "k", 9, 0, 0.0, &op) == 2);
  // concurrency
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([p, t] {
      int o;
      std::string id = "job" + std::to_string(t % 3);
      int par = 1;
      for (int i = 0; i < 2000; ++i) par = kml_policy_decide(p, id.c_str(), 2, par, 1.0 + (i % 7) * 0.1, &o);
      kml_policy_finish(p, id.c_str());
    });
  for (auto& t : ts) t.join();
  kml_policy_free(p);
}

static void test_merger() {
  const long long n = 100003;
  std::vector<std::vector<float>> bufs(5, std::vector<float>(n));
  std::vector<const float*> ptrs;
  for (int k = 0; k < 5; ++k) {
    for (long long i = 0; i < n; ++i) bufs[k][i] = (float)(k + 1) * 0.5f + (float)(i % 13);
    ptrs.push_back(bufs[k].data());
  }
  std::vector<float> out(n);
  CHECK(kml_sum_f32(out.data(), ptrs.data(), 5, n, 4) == 0);
  for (long long i = 0; i < n; i += 997) CHECK(std::fabs(out[i] - (7.5f + 5.0f * (float)(i % 13))) < 1e-4f);
  CHECK(kml_average_f32(out.data(), ptrs.data(), 5, n, 3) == 0);
  for (long long i = 0; i < n; i += 991) CHECK(std::fabs(out[i] - (1.5f + (float)(i % 13))) < 1e-4f);
  std::vector<float> acc(n, 1.0f);
  CHECK(kml_accumulate_f32(acc.data(), bufs[0].data(), n) == 0);
  CHECK(std::fabs(acc[5] - (1.0f + bufs[0][5])) < 1e-6f);
}

static void write_npy(const char* path, int rows, int cols) {
  FILE* f = std::fopen(path, "wb");
  char hdr[128];
  int len = std::snprintf(hdr, sizeof hdr, "{'descr': '<f4', 'fortran_order': False, 'shape': (%d, %d), }", rows,
                          cols);
  int total = 10 + len + 1;
  int pad = (64 - total % 64) % 64;
  unsigned short hl = (unsigned short)(len + pad + 1);
  std::fwrite("\x93NUMPY\x01\x00", 1, 8, f);
  std::fwrite(&hl, 2, 1, f);
  std::fwrite(hdr, 1, len, f);
  for (int i = 0; i < pad; ++i) std::fputc(' ', f);
  std::fputc('\n', f);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
      float v = (float)(r * 1000 + c);
      std::fwrite(&v, 4, 1, f);
    }
  std::fclose(f);
}

static void test_npy(const char* dir) {
  std::string path = std::string(dir) + "/rt_test.npy";
  write_npy(path.c_str(), 300, 7);
  void* h = kml_npy_open(path.c_str());
  CHECK(h != nullptr);
  if (!h) return;
  long long info[16] = {0};
  CHECK(kml_npy_info(h, info) == 0);
  std::vector<float> dst(50 * 7);
  CHECK(kml_npy_gather(h, 100, 50, dst.data(), 4) == 0);
  CHECK(dst[0] == 100000.0f && dst[7 * 49 + 6] == 149006.0f);
  CHECK(kml_npy_gather(h, 290, 50, dst.data(), 2) != 0);  // out of range must be rejected
  kml_npy_close(h);
  CHECK(kml_npy_open((path + ".missing").c_str()) == nullptr);
}

// prefetcher: ranges pushed ahead are filled by the background thread into a small ring
// and taken in order, byte-exact; more ranges than slots exercises slot recycling; free
// with ranges still queued must not hang or leak
static void test_prefetch(const char* dir) {
  std::string path = std::string(dir) + "/rt_prefetch.npy";
  write_npy(path.c_str(), 1000, 5);
  void* h = kml_npy_open(path.c_str());
  CHECK(h != nullptr);
  if (!h) return;
  void* pf = kml_prefetch_new(h, 3, 64);
  CHECK(pf != nullptr);
  CHECK(kml_prefetch_push(pf, 0, 65) == -1);      // larger than a slot
  CHECK(kml_prefetch_push(pf, 990, 20) == -2);    // out of range
  std::vector<long long> r0s;
  for (long long r = 0; r + 64 <= 1000; r += 64) {
    CHECK(kml_prefetch_push(pf, r, 64) >= 0);
    r0s.push_back(r);
  }
  CHECK(kml_prefetch_push(pf, 960, 40) >= 0);
  r0s.push_back(960);
  CHECK(kml_prefetch_pending(pf) == (long long)r0s.size());
  std::vector<float> dst(64 * 5);
  for (size_t i = 0; i < r0s.size(); ++i) {
    const long long n = kml_prefetch_take_host(pf, dst.data());
    CHECK(n == (r0s[i] == 960 ? 40 : 64));
    bool ok = true;
    for (long long k = 0; k < n && ok; ++k)
      for (int c = 0; c < 5; ++c)
        ok = ok && dst[k * 5 + c] == (float)((r0s[i] + k) * 1000 + c);
    CHECK(ok);
  }
  CHECK(kml_prefetch_take_host(pf, dst.data()) == -1);   // nothing left
  for (int i = 0; i < 6; ++i) kml_prefetch_push(pf, 64 * i, 64);
  (void)kml_prefetch_take_host(pf, dst.data());
  kml_prefetch_free(pf);                                  // 5 still queued
  kml_npy_close(h);
}

// the fill thread against a producer thread pushing ranges, a consumer thread taking them in
// order (byte-exact), and a thread polling pending() — the interleavings ThreadSanitizer watches —
// then free() racing the fill thread with ranges still queued, several times over
static void test_prefetch_concurrent(const char* dir) {
  std::string path = std::string(dir) + "/rt_prefetch_mt.npy";
  const int rows = 4000, cols = 3;
  write_npy(path.c_str(), rows, cols);
  void* h = kml_npy_open(path.c_str());
  CHECK(h != nullptr);
  if (!h) return;
  for (int round = 0; round < 4; ++round) {
    void* pf = kml_prefetch_new(h, 2 + round, 32);
    CHECK(pf != nullptr);
    const int nranges = 120;
    std::atomic<int> pushed{0};
    std::atomic<bool> done{false};
    std::atomic<int> bad{0};
    std::thread producer([&] {
      for (int i = 0; i < nranges; ++i) {
        const long long r0 = (i * 37LL) % (rows - 32);
        if (kml_prefetch_push(pf, r0, 1 + i % 32) < 0) bad.fetch_add(1);
        pushed.fetch_add(1);
        if (i % 7 == 0) std::this_thread::yield();
      }
    });
    std::thread consumer([&] {
      std::vector<float> dst(32 * cols);
      for (int i = 0; i < nranges; ++i) {
        while (pushed.load() <= i) std::this_thread::yield();
        const long long n = kml_prefetch_take_host(pf, dst.data());
        const long long r0 = (i * 37LL) % (rows - 32);
        if (n != 1 + i % 32) { bad.fetch_add(1); continue; }
        for (long long k = 0; k < n; ++k)
          for (int c = 0; c < cols; ++c)
            if (dst[k * cols + c] != (float)((r0 + k) * 1000 + c)) bad.fetch_add(1);
      }
      done.store(true);
    });
    std::thread monitor([&] {
      while (!done.load()) {
        const long long p = kml_prefetch_pending(pf);
        if (p < 0 || p > nranges) bad.fetch_add(1);
        std::this_thread::yield();
      }
    });
    producer.join();
    consumer.join();
    monitor.join();
    CHECK(bad.load() == 0);
    for (int i = 0; i < 5; ++i) kml_prefetch_push(pf, 32 * i, 32);   // queued when freed
    kml_prefetch_free(pf);
  }
  kml_npy_close(h);
}

int main(int argc, char** argv) {
  test_policy();
  test_merger();
  test_npy(argc > 1 ? argv[1] : "/tmp");
  test_prefetch(argc > 1 ? argv[1] : "/tmp");
  test_prefetch_concurrent(argc > 1 ? argv[1] : "/tmp");
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("runtime host tests OK\n");
  return 0;
}
