// Device-memory cache of one plan: the buffers of its batches and their training state.
//
// The training input pipeline (ignnition_amd/training.py BatchPrefetcher) builds the next batches
// on worker threads while the GPU runs the current step.  Straight hipMalloc / hipFree there cost
// more than the step itself: hipMalloc serialises across threads and hipFree waits for the device.
// Batches of one workload have near-identical shapes, so their blocks are cached by size class and
// handed to the next batch.  A returned block carries an event recorded on the plan stream when
// its batch was destroyed; it is reused only once that event has completed, so no kernel still in
// flight can see its memory change.  Size classes keep 3 significant bits (<= 12.5% slack).
//
// IGN_POOL=0 bypasses the cache (hipMalloc / hipFree per block).  IGN_POOL_POISON=1 fills every
// scratch block it hands out with NaN (0xFF bytes): the parity tests under it show that no kernel
// reads batch scratch it has not written (tests/test_gpu_parity.py).  The idle bytes are capped per
// device across every pool of the process (one per plan: bench's sub-batch engines, a trainer's eval
// engine): IGN_POOL_CACHE_GB, default half the device memory free when the first pool was created;
// ign_plan_trim_cache releases a plan's.  The cache is trimmed to the cap by the allocating threads
// (a training loop's batch builders), never by a release: hipFree waits for the device, and a
// release is the training step's own Batch.close.  When hipMalloc runs out of memory, every pool of
// the device gives its idle blocks back before the retry, not only the allocating plan's.
//
// The host side has the same problem: the batch builders' index tables are ~10^8 bytes of host
// memory per batch.  hvec (engine_internal.h) draws blocks >= 1 MiB from a process-wide cache
// (IGN_HOST_CACHE_GB idle bytes kept, default 4) whose blocks keep their pages and are pinned,
// so the uploads from them are direct DMA.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "engine_internal.h"

namespace ign {

namespace {

struct Fence {
  hipEvent_t ev = nullptr;
  bool done = false;
  ~Fence() {
    if (ev) hipEventDestroy(ev);
  }
  bool ready() {
    if (!done && (!ev || hipEventQuery(ev) == hipSuccess)) done = true;
    return done;
  }
};

size_t size_class(size_t bytes) {
  if (bytes <= 4096) return 4096;
  int top = 63 - __builtin_clzll(bytes);        // 2^top <= bytes
  size_t step = (size_t)1 << (top - 2);         // 4 classes per octave
  return (bytes + step - 1) / step * step;
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// the idle-byte budget of one device, shared by every pool of the process on it
struct DeviceBudget {
  std::atomic<int64_t> idle{0};
  size_t cap = 0;
};

struct Registry {
  std::mutex mu;
  std::map<int, DeviceBudget> budgets;              // std::map: stable addresses
  std::vector<std::weak_ptr<DevPool>> pools;
};
Registry& registry() {
  static Registry* r = new Registry();   // never destroyed: pools may outlive static destruction order
  return *r;
}

}  // namespace

struct DevPool {
  struct Idle {
    void* ptr;
    std::shared_ptr<Fence> fence;
  };
  std::mutex mu;
  std::map<size_t, std::vector<Idle>> idle;    // by size class, oldest first
  std::unordered_map<void*, size_t> live;      // block -> size class
  size_t idle_bytes = 0;
  DeviceBudget* budget = nullptr;
  bool enabled = true, poison = false;
  int device = 0;

  void add_idle(size_t cls) {
    idle_bytes += cls;
    budget->idle += (int64_t)cls;
  }
  void sub_idle(size_t cls) {
    idle_bytes -= cls;
    budget->idle -= (int64_t)cls;
  }

  // free idle blocks whose fence has completed, oldest classes' first, until idle_bytes <= target;
  // with wait, also those still in flight (their fences are waited for).  With out, the blocks are
  // only taken out of the cache and handed back for the caller to hipFree once it has dropped the
  // lock (hipFree waits for the device: under the lock it stalled every other thread's release)
  void trim(size_t target, bool wait, std::vector<void*>* out = nullptr) {
    for (auto it = idle.begin(); it != idle.end() && idle_bytes > target;) {
      auto& v = it->second;
      for (size_t i = 0; i < v.size() && idle_bytes > target;) {
        if (wait && v[i].fence->ev) hipEventSynchronize(v[i].fence->ev);
        if (v[i].fence->ready()) {
          if (out) out->push_back(v[i].ptr);
          else hipFree(v[i].ptr);
          sub_idle(it->first);
          v.erase(v.begin() + i);
        } else {
          ++i;
        }
      }
      it = v.empty() ? idle.erase(it) : std::next(it);
    }
  }

  ~DevPool() {
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(device);
    trim(0, true);
    hipSetDevice(prev);
  }
};

std::shared_ptr<DevPool> pool_create(int device) {
  auto pool = std::make_shared<DevPool>();
  pool->device = device;
  pool->enabled = env_int("IGN_POOL", 1) != 0;
  pool->poison = env_int("IGN_POOL_POISON", 0) != 0;
  Registry& reg = registry();
  std::lock_guard<std::mutex> g(reg.mu);
  auto found = reg.budgets.find(device);
  if (found == reg.budgets.end()) {
    // the device's cap, once: half its memory free now (round 5 kept half the TOTAL memory per pool,
    // so several plans could together cache more than the device has).  A training batch of 512 x
    // synth50 holds ~11 GB of device blocks and the input pipeline keeps workers + 1 of them in
    // flight.  Under a 16 GB cap every release trimmed blocks with hipFree -- which waits for the
    // device -- in the step's own Batch.close (22 -> 57 ms per step, round 5); a quarter of the free
    // memory still did once the cache had filled (close 17 ms per step at 8 input workers, 62 at 12,
    // r06_c15).  Releases no longer trim (pool_alloc does)
    DeviceBudget& b = reg.budgets[device];
    const int gb = env_int("IGN_POOL_CACHE_GB", -1);
    size_t free_b = 0, total_b = 0;
    int prev = 0;
    hipGetDevice(&prev);
    if (hipSetDevice(device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess) b.cap = free_b / 2;
    else b.cap = (size_t)16 << 30;
    hipSetDevice(prev);
    if (gb >= 0) b.cap = (size_t)gb << 30;
    found = reg.budgets.find(device);
  }
  pool->budget = &found->second;
  // drop expired entries while here
  auto& v = reg.pools;
  v.erase(std::remove_if(v.begin(), v.end(), [](const std::weak_ptr<DevPool>& w) { return w.expired(); }), v.end());
  v.push_back(pool);
  return pool;
}

namespace {

// the other live pools of a device (their idle blocks are given back on OOM or over the budget)
std::vector<std::shared_ptr<DevPool>> device_pools(int device, const DevPool* except) {
  Registry& reg = registry();
  std::lock_guard<std::mutex> g(reg.mu);
  std::vector<std::shared_ptr<DevPool>> out;
  for (auto& w : reg.pools)
    if (auto p = w.lock())
      if (p.get() != except && p->device == device) out.push_back(std::move(p));
  return out;
}

// free idle blocks of the device's other pools until its idle bytes are within `target`
// (each pool under its own lock, never two at once; wait: also blocks still in flight)
void trim_device(DevPool* self, size_t target, bool wait) {
  for (auto& p : device_pools(self->device, self)) {
    if (self->budget->idle.load() <= (int64_t)target) return;
    std::vector<void*> victims;
    {
      std::lock_guard<std::mutex> g(p->mu);
      const int64_t excess = p->budget->idle.load() - (int64_t)target;
      if (excess <= 0) return;
      p->trim(p->idle_bytes > (size_t)excess ? p->idle_bytes - (size_t)excess : 0, wait, &victims);
    }
    for (void* v : victims) hipFree(v);
  }
}

}  // namespace

bool pool_enabled(const DevPool* pool) { return pool && pool->enabled; }

hipError_t pool_alloc(DevPool* pool, void** out, size_t bytes, bool scratch) {
  *out = nullptr;
  if (!pool->enabled) {
    hipError_t e = hipMalloc(out, bytes);
    if (e == hipSuccess && scratch && pool->poison) e = hipMemsetAsync(*out, 0xFF, bytes, upload_stream());
    return e;
  }
  const size_t cls = size_class(bytes);
  {
    // a ready block of this size class or of the next two (<= 1.5x the request): batches of one
    // workload differ a little in size, and blocks stranded one class up would fill the cache
    std::lock_guard<std::mutex> g(pool->mu);
    auto it = pool->idle.lower_bound(cls);
    for (int tried = 0; !*out && it != pool->idle.end() && tried < 3 && it->first * 2 <= cls * 3; ++tried) {
      auto& v = it->second;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].fence->ready()) {
          *out = v[i].ptr;
          v.erase(v.begin() + i);
          pool->sub_idle(it->first);
          pool->live[*out] = it->first;
          break;
        }
      it = v.empty() ? pool->idle.erase(it) : std::next(it);
    }
  }
  if (!*out) {
    hipError_t e = hipMalloc(out, cls);
    // out of memory: give back the device's idle blocks and retry -- first those whose fence has
    // completed, then (still short) every one, waiting for the in-flight fences.  The blocks are freed
    // after the lock is dropped: the step's own release takes this lock, and hipFree / the fence waits
    // under it stalled the step for the whole trim (10-12 ms per step with 10-12 input workers, r06_c11)
    for (int pass = 0; e == hipErrorOutOfMemory && pass < 2; ++pass) {
      (void)hipGetLastError();
      static const bool prof = env_int("IGN_BUILD_PROF", 0) != 0;
      if (prof)
        fprintf(stderr, "[ign-pool] out of memory for a %.1f MB block: trimming the device's idle blocks (%s)\n",
                cls / 1048576.0, pass ? "waiting for in-flight ones" : "completed ones");
      std::vector<void*> victims;
      if (pass == 1) {   // the in-flight fences, waited for outside the lock
        std::vector<std::shared_ptr<Fence>> fences;
        {
          std::lock_guard<std::mutex> g(pool->mu);
          for (auto& kv : pool->idle)
            for (auto& b : kv.second)
              if (!b.fence->done && b.fence->ev) fences.push_back(b.fence);
        }
        for (auto& f : fences) hipEventSynchronize(f->ev);
      }
      {
        std::lock_guard<std::mutex> g(pool->mu);
        pool->trim(0, false, &victims);
      }
      for (void* v : victims) hipFree(v);
      trim_device(pool, 0, pass == 1);
      e = hipMalloc(out, cls);
    }
    if (e != hipSuccess) {
      *out = nullptr;
      return e;
    }
    std::lock_guard<std::mutex> g(pool->mu);
    pool->live[*out] = cls;
  }
  // over the device's budget: this pool's own idle blocks first, then the other pools' (completed
  // fences only; freed here, on the allocating thread, outside the lock)
  if (pool->budget->idle.load() > (int64_t)pool->budget->cap) {
    std::vector<void*> victims;
    {
      std::lock_guard<std::mutex> g(pool->mu);
      const int64_t excess = pool->budget->idle.load() - (int64_t)pool->budget->cap;
      if (excess > 0) pool->trim(pool->idle_bytes > (size_t)excess ? pool->idle_bytes - (size_t)excess : 0, false, &victims);
    }
    for (void* v : victims) hipFree(v);
    if (pool->budget->idle.load() > (int64_t)pool->budget->cap) trim_device(pool, pool->budget->cap, false);
  }
  if (scratch && pool->poison) return hipMemsetAsync(*out, 0xFF, bytes, upload_stream());
  return hipSuccess;
}

void pool_release(DevPool* pool, const std::vector<void*>& blocks, hipStream_t after) {
  if (blocks.empty()) return;
  if (!pool->enabled) {
    if (after) hipStreamSynchronize(after);
    for (void* b : blocks) hipFree(b);
    return;
  }
  auto fence = std::make_shared<Fence>();
  if (hipEventCreateWithFlags(&fence->ev, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(fence->ev, after) != hipSuccess) {
    if (fence->ev) hipEventDestroy(fence->ev);
    fence->ev = nullptr;
    if (after) hipStreamSynchronize(after);
  }
  {
    std::lock_guard<std::mutex> g(pool->mu);
    for (void* b : blocks) {
      auto it = pool->live.find(b);
      if (it == pool->live.end()) continue;   // not ours (cannot happen): leave it alone
      const size_t cls = it->second;
      pool->live.erase(it);
      pool->idle[cls].push_back({b, fence});
      pool->add_idle(cls);
    }
  }
}

// ---- host blocks ----------------------------------------------------------------------------
namespace {

struct HostCache {
  std::mutex mu;
  std::map<size_t, std::vector<void*>> idle;   // by size class
  std::unordered_map<void*, bool> pinned;      // every live or idle block -> registered for DMA
  std::unordered_map<void*, size_t> cls_of;    // every live or idle block -> its size class
  size_t idle_bytes = 0, live_bytes = 0;
  size_t cap = 0;
  int64_t n_map = 0, n_unmap = 0;   // IGN_BUILD_PROF: blocks mapped + pinned, and unpinned + unmapped
  HostCache() { cap = (size_t)std::max(0, env_int("IGN_HOST_CACHE_GB", 4)) << 30; }
  void unmap(void* p, size_t cls) {
    auto it = pinned.find(p);
    if (it != pinned.end()) {
      if (it->second) hipHostUnregister(p);
      pinned.erase(it);
    }
    cls_of.erase(p);
    munmap(p, cls);
    n_unmap++;
  }
};

HostCache& host_cache() {
  static HostCache* c = new HostCache();   // never destroyed: blocks may be freed during exit
  return *c;
}

size_t host_class(size_t bytes) {
  const size_t two_mb = (size_t)2 << 20;
  return std::max(size_class(bytes), (bytes + two_mb - 1) / two_mb * two_mb);
}

}  // namespace

void* host_block_alloc(size_t bytes) {
  HostCache& c = host_cache();
  const size_t cls = host_class(bytes);
  {
    // an idle block of this class or of the next two (<= 1.5x): batches of one workload differ a
    // little in size, and a miss maps and pins a new block (page faults + registration: the index
    // tables' first MP took 12 -> 28 ms over four batches as blocks stranded one class up)
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.idle.lower_bound(cls);
    for (int tried = 0; it != c.idle.end() && tried < 3 && it->first * 2 <= cls * 3; ++tried, ++it)
      if (!it->second.empty()) {
        void* p = it->second.back();
        it->second.pop_back();
        c.idle_bytes -= it->first;
        c.live_bytes += it->first;
        return p;
      }
  }
  void* p = mmap(nullptr, cls, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  madvise(p, cls, MADV_HUGEPAGE);
  // pinned: hipMemcpyAsync from it is a direct DMA instead of a staged copy (best effort: the
  // block works as pageable memory when registration is refused)
  const bool reg = hipHostRegister(p, cls, hipHostRegisterPortable) == hipSuccess;
  if (!reg) (void)hipGetLastError();
  std::lock_guard<std::mutex> g(c.mu);
  c.pinned[p] = reg;
  c.cls_of[p] = cls;
  c.live_bytes += cls;
  c.n_map++;
  return p;
}

void host_block_free(void* p, size_t bytes) {
  if (!p) return;
  HostCache& c = host_cache();
  std::lock_guard<std::mutex> g(c.mu);
  auto k = c.cls_of.find(p);
  const size_t cls = k != c.cls_of.end() ? k->second : host_class(bytes);   // (a block may be one class up)
  c.idle[cls].push_back(p);
  c.idle_bytes += cls;
  c.live_bytes -= cls;
  // over the cap: unmap idle blocks, largest classes first
  for (auto it = c.idle.rbegin(); c.idle_bytes > c.cap && it != c.idle.rend(); ++it)
    while (c.idle_bytes > c.cap && !it->second.empty()) {
      c.unmap(it->second.back(), it->first);
      it->second.pop_back();
      c.idle_bytes -= it->first;
    }
}

void pool_trim_idle(DevPool* pool) {
  if (!pool) return;
  std::lock_guard<std::mutex> g(pool->mu);
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(pool->device);
  pool->trim(0, true);
  hipSetDevice(prev);
}

void host_cache_trim() {
  HostCache& c = host_cache();
  std::lock_guard<std::mutex> g(c.mu);
  for (auto& kv : c.idle) {
    for (void* p : kv.second) c.unmap(p, kv.first);
    c.idle_bytes -= kv.first * kv.second.size();
    kv.second.clear();
  }
}

void host_cache_stats(int64_t* live, int64_t* idle, int64_t* maps, int64_t* unmaps) {
  HostCache& c = host_cache();
  std::lock_guard<std::mutex> g(c.mu);
  *live = (int64_t)c.live_bytes;
  *idle = (int64_t)c.idle_bytes;
  *maps = c.n_map;
  *unmaps = c.n_unmap;
}

void pool_stats(DevPool* pool, int64_t* live_bytes, int64_t* idle_bytes) {
  std::lock_guard<std::mutex> g(pool->mu);
  int64_t l = 0;
  for (auto& kv : pool->live) l += (int64_t)kv.second;
  if (live_bytes) *live_bytes = l;
  if (idle_bytes) *idle_bytes = (int64_t)pool->idle_bytes;
}

}  // namespace ign
