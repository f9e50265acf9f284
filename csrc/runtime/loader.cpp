// loader.cpp — native data path: .npy shard reader, pinned staging ring, async H2D.
//
// The reference streams datasets from MongoDB: every 64-sample document is a pickled
// ndarray that the function unpickles and vstacks (python/kubeml/kubeml/dataset.py:184-223).
// Here a dataset split is ONE contiguous .npy file (written by the storage service,
// kubeml_amd/store/shards.py) that is memory-mapped; a "document" i is just rows
// [64 i, 64 (i+1)).  Loading a document range is a bounds-checked pointer range, and
// moving it to the GPU goes through a ring of pinned (hipHostMalloc) buffers filled by
// a background thread and drained with hipMemcpyAsync on the caller's stream, so
// host copies overlap device work and never touch pageable memory on the DMA path.
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#define KML_API extern "C" __attribute__((visibility("default")))

namespace {

struct Npy {
  int fd = -1;
  void* map = nullptr;
  size_t map_len = 0;
  const uint8_t* data = nullptr;
  size_t nbytes = 0;
  int ndim = 0;
  long long shape[8] = {0};
  int itemsize = 0;
  char kind = 0;  // 'u','i','f','b'
  long long row_bytes = 0;
};

// minimal NPY v1/v2/v3 header parser (C-order, little-endian numeric dtypes only)
bool parse_header(const char* h, size_t len, Npy* n) {
  std::string s(h, len);
  auto d = s.find("'descr'");
  if (d == std::string::npos) return false;
  auto q1 = s.find('\'', d + 7);
  auto q2 = s.find('\'', q1 + 1);
  if (q1 == std::string::npos || q2 == std::string::npos) return false;
  std::string descr = s.substr(q1 + 1, q2 - q1 - 1);  // e.g. "<f4", "|u1"
  if (descr.size() < 3) return false;
  if (descr[0] == '>') return false;
  n->kind = descr[1];
  n->itemsize = std::atoi(descr.c_str() + 2);
  if (s.find("'fortran_order': True") != std::string::npos) return false;
  auto sp = s.find("'shape'");
  auto p1 = s.find('(', sp);
  auto p2 = s.find(')', p1);
  if (sp == std::string::npos || p1 == std::string::npos || p2 == std::string::npos) return false;
  std::string dims = s.substr(p1 + 1, p2 - p1 - 1);
  n->ndim = 0;
  size_t i = 0;
  while (i < dims.size() && n->ndim < 8) {
    while (i < dims.size() && (dims[i] == ' ' || dims[i] == ',')) ++i;
    if (i >= dims.size()) break;
    n->shape[n->ndim++] = std::atoll(dims.c_str() + i);
    while (i < dims.size() && dims[i] != ',') ++i;
  }
  long long rb = n->itemsize;
  for (int k = 1; k < n->ndim; ++k) rb *= n->shape[k];
  n->row_bytes = rb;
  return true;
}

struct Slot {
  void* host = nullptr;
  bool pinned = false;  // hipHostMalloc'd (else malloc fallback: no GPU runtime)
  size_t cap = 0;
  long long row0 = 0, nrows = 0;
  int state = 0;  // 0 free, 1 filling, 2 ready, 3 in flight (H2D queued)
  hipEvent_t ev = nullptr;
};

struct Prefetcher {
  Npy* src = nullptr;
  std::vector<Slot> slots;
  std::vector<std::pair<long long, long long>> ranges;  // (row0, nrows) in order
  size_t next_fill = 0, next_take = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::thread th;
  std::atomic<bool> stop{false};
};

void fill_loop(Prefetcher* p) {
  for (;;) {
    size_t idx;
    long long r0, nr;
    Slot* s = nullptr;
    {
      std::unique_lock<std::mutex> lk(p->mu);
      p->cv.wait(lk, [&] {
        if (p->stop) return true;
        if (p->next_fill >= p->ranges.size()) return false;
        Slot& c = p->slots[p->next_fill % p->slots.size()];
        return c.state == 0 || c.state == 3;
      });
      if (p->stop) return;
      idx = p->next_fill++;
      s = &p->slots[idx % p->slots.size()];
      if (s->state == 3) {
        // slot still owned by an H2D copy: wait for it here, off the caller's thread
        // (the consumer never has to recycle slots, so take() cannot deadlock on it)
        hipEvent_t ev = s->ev;
        lk.unlock();
        if (ev) (void)hipEventSynchronize(ev);
        lk.lock();
      }
      s->state = 1;
      r0 = p->ranges[idx].first;
      nr = p->ranges[idx].second;
    }
    const size_t bytes = (size_t)nr * p->src->row_bytes;
    std::memcpy(s->host, p->src->data + (size_t)r0 * p->src->row_bytes, bytes);
    {
      std::lock_guard<std::mutex> lk(p->mu);
      s->row0 = r0;
      s->nrows = nr;
      s->state = 2;
    }
    p->cv.notify_all();
  }
}

}  // namespace

KML_API void* kml_npy_open(const char* path) {
  Npy* n = new Npy();
  n->fd = ::open(path, O_RDONLY);
  if (n->fd < 0) { delete n; return nullptr; }
  struct stat st;
  if (fstat(n->fd, &st) != 0 || st.st_size < 16) { ::close(n->fd); delete n; return nullptr; }
  n->map_len = (size_t)st.st_size;
  n->map = mmap(nullptr, n->map_len, PROT_READ, MAP_SHARED, n->fd, 0);
  if (n->map == MAP_FAILED) { ::close(n->fd); delete n; return nullptr; }
  const uint8_t* b = static_cast<const uint8_t*>(n->map);
  if (std::memcmp(b, "\x93NUMPY", 6) != 0) { munmap(n->map, n->map_len); ::close(n->fd); delete n; return nullptr; }
  const int major = b[6];
  size_t hlen, hoff;
  if (major == 1) { hlen = b[8] | (b[9] << 8); hoff = 10; }
  else { hlen = b[8] | (b[9] << 8) | (b[10] << 16) | ((size_t)b[11] << 24); hoff = 12; }
  if (!parse_header(reinterpret_cast<const char*>(b + hoff), hlen, n)) {
    munmap(n->map, n->map_len); ::close(n->fd); delete n; return nullptr;
  }
  n->data = b + hoff + hlen;
  n->nbytes = n->map_len - hoff - hlen;
  madvise(n->map, n->map_len, MADV_SEQUENTIAL);
  return n;
}

KML_API void kml_npy_close(void* h) {
  Npy* n = static_cast<Npy*>(h);
  if (!n) return;
  munmap(n->map, n->map_len);
  ::close(n->fd);
  delete n;
}

// info: [ndim, itemsize, kind(char), row_bytes, shape0..shape7]
KML_API int kml_npy_info(void* h, long long* info) {
  Npy* n = static_cast<Npy*>(h);
  info[0] = n->ndim; info[1] = n->itemsize; info[2] = n->kind; info[3] = n->row_bytes;
  for (int i = 0; i < 8; ++i) info[4 + i] = n->shape[i];
  return 0;
}

KML_API const void* kml_npy_data(void* h) { return static_cast<Npy*>(h)->data; }

// copy rows [row0, row0+nrows) into dst (host memory), split across threads
KML_API int kml_npy_gather(void* h, long long row0, long long nrows, void* dst, int threads) {
  Npy* n = static_cast<Npy*>(h);
  if (row0 < 0 || nrows < 0 || row0 + nrows > n->shape[0]) return 1;
  const size_t bytes = (size_t)nrows * n->row_bytes;
  const uint8_t* src = n->data + (size_t)row0 * n->row_bytes;
  if (threads <= 1 || bytes < (1u << 20)) { std::memcpy(dst, src, bytes); return 0; }
  std::vector<std::thread> ts;
  const size_t per = (bytes + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t o = t * per;
    if (o >= bytes) break;
    const size_t l = std::min(per, bytes - o);
    ts.emplace_back([=] { std::memcpy(static_cast<uint8_t*>(dst) + o, src + o, l); });
  }
  for (auto& t : ts) t.join();
  return 0;
}

KML_API void* kml_pinned_alloc(long long bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

KML_API void kml_pinned_free(void* p) { if (p) (void)hipHostFree(p); }

KML_API int kml_h2d_async(void* dst_dev, const void* src_host, long long bytes, hipStream_t s) {
  return (int)hipMemcpyAsync(dst_dev, src_host, (size_t)bytes, hipMemcpyHostToDevice, s);
}

// ---- prefetcher: ranges of rows staged through a pinned ring by a background thread ----

KML_API void* kml_prefetch_new(void* npy, int nslots, long long max_rows) {
  Npy* n = static_cast<Npy*>(npy);
  Prefetcher* p = new Prefetcher();
  p->src = n;
  p->slots.resize(nslots < 2 ? 2 : nslots);
  for (auto& s : p->slots) {
    s.cap = (size_t)max_rows * n->row_bytes;
    s.pinned = hipHostMalloc(&s.host, s.cap, hipHostMallocDefault) == hipSuccess;
    if (!s.pinned) s.host = malloc(s.cap);
    if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) s.ev = nullptr;
  }
  p->th = std::thread(fill_loop, p);
  return p;
}

// queue a row range (in order); returns its sequence number
KML_API long long kml_prefetch_push(void* h, long long row0, long long nrows) {
  Prefetcher* p = static_cast<Prefetcher*>(h);
  if (nrows * p->src->row_bytes > (long long)p->slots[0].cap) return -1;
  if (row0 < 0 || row0 + nrows > p->src->shape[0]) return -2;
  long long id;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    id = (long long)p->ranges.size();
    p->ranges.emplace_back(row0, nrows);
  }
  p->cv.notify_all();
  return id;
}

namespace {

// wait for the next range in order; returns its slot (state stays 2 until released)
Slot* wait_ready(Prefetcher* p) {
  std::unique_lock<std::mutex> lk(p->mu);
  if (p->next_take >= p->ranges.size()) return nullptr;
  Slot* slot = &p->slots[p->next_take % p->slots.size()];
  p->cv.wait(lk, [&] { return slot->state == 2 || p->stop; });
  if (p->stop) return nullptr;
  p->next_take++;
  return slot;
}

}  // namespace

// take the next ready range and copy it to dst_dev on stream s; returns rows copied.
// The slot is handed back to the fill thread as "in flight" (state 3): the fill thread
// waits for the copy's event before overwriting it.
KML_API long long kml_prefetch_take(void* h, void* dst_dev, hipStream_t s) {
  Prefetcher* p = static_cast<Prefetcher*>(h);
  Slot* slot = wait_ready(p);
  if (!slot) return -1;
  const size_t bytes = (size_t)slot->nrows * p->src->row_bytes;
  if (hipMemcpyAsync(dst_dev, slot->host, bytes, hipMemcpyHostToDevice, s) != hipSuccess) return -3;
  if (slot->ev) hipEventRecord(slot->ev, s);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    slot->state = slot->ev ? 3 : 0;
  }
  p->cv.notify_all();
  return slot->nrows;
}

// host-destination take (CPU workers, host tests): synchronous memcpy, slot freed at once
KML_API long long kml_prefetch_take_host(void* h, void* dst) {
  Prefetcher* p = static_cast<Prefetcher*>(h);
  Slot* slot = wait_ready(p);
  if (!slot) return -1;
  std::memcpy(dst, slot->host, (size_t)slot->nrows * p->src->row_bytes);
  const long long n = slot->nrows;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    slot->state = 0;
  }
  p->cv.notify_all();
  return n;
}

// ranges pushed but not yet taken
KML_API long long kml_prefetch_pending(void* h) {
  Prefetcher* p = static_cast<Prefetcher*>(h);
  std::lock_guard<std::mutex> lk(p->mu);
  return (long long)(p->ranges.size() - p->next_take);
}

KML_API void kml_prefetch_free(void* h) {
  Prefetcher* p = static_cast<Prefetcher*>(h);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    p->stop = true;
  }
  p->cv.notify_all();
  if (p->th.joinable()) p->th.join();
  for (auto& s : p->slots) {
    if (s.ev) { hipEventSynchronize(s.ev); hipEventDestroy(s.ev); }
    if (s.host && s.pinned) (void)hipHostFree(s.host);
    else free(s.host);
  }
  delete p;
}
