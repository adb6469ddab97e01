// engine.cpp — C ABI (include/ignmp.h), plan lowering, native batch builder, forward driver.
//
// Reference behaviour restated here (generate_model.py = GM, auxilary_classes.py = AUX):
//  * hidden-state init per entity                                  GM:396-400, AUX:128-160
//  * T iterations x stages x MPs, destination state overwritten
//    after each MP (later MPs of a stage see it)                   GM:406-603
//  * per-graph dense padding semantics of the combine step:
//      lens = in-degree, Lmax = max(seq)+1 per graph and source,
//      source k's slots start after sources 0..k-1's Lmax           GM:477-543
//      interleave permutes slots through indices_<src>_to_<dst>    AUX:421-440, GM:507-519
//      sorted update consumes positions 0..final_len-1 (holes are
//      zero inputs, later positions dropped)                       AUX:767-796
//    These become per-destination step tables (CSR) built here on the host, once per batch.
//  * readout predict op (Dense stack)                              GM:611-629
// Errors the reference raises at run time (e.g. gather_nd(-1) when final_len = 0, scatter_nd
// with an out-of-range interleave index, an adjacency with no edges) are returned as
// IGN_ERR_INVALID with a message.

#include <hip/hip_runtime.h>

#include <atomic>
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ignmp.h"
#include "kernels.h"

#include "engine_internal.h"
#include "train_kernels.h"

namespace ign {


thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}


int set_device(int dev) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(IGN_ERR_DEVICE, "no HIP device available (%s)", e == hipSuccess ? "0 devices" : hipGetErrorString(e));
  if (dev < 0 || dev >= n) return fail(IGN_ERR_DEVICE, "device %d out of range (%d devices)", dev, n);
  HIP_TRY(hipSetDevice(dev));
  return IGN_OK;
}

int ensure_device(ign_plan* p) {
  int rc = set_device(p->device);
  if (rc) return rc;
  if (!p->stream && !p->external_stream) {
    HIP_TRY(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    p->own_stream = true;
  }
  if (!p->d_params) {
    HIP_TRY(hipMalloc(&p->d_params, std::max<int64_t>(p->n_params, 1) * sizeof(float)));
    HIP_TRY(hipMalloc(&p->d_packed, std::max<int64_t>(p->n_packed, 1) * sizeof(float)));
    // on the plan stream and waited for: a null-stream memset is not ordered with the
    // non-blocking plan stream and could land after ign_plan_set_params' copy
    HIP_TRY(hipMemsetAsync(p->d_params, 0, std::max<int64_t>(p->n_params, 1) * sizeof(float), p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
  }
  if (!p->pool) p->pool = pool_create(p->device);
  return IGN_OK;
}

// one non-blocking upload stream per host thread and device (a stream belongs to the device that
// was current when it was created; a thread may build batches for plans on several devices)
hipStream_t upload_stream() {
  thread_local std::vector<hipStream_t> streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if ((int)streams.size() <= dev) streams.resize(dev + 1, nullptr);
  hipStream_t& s = streams[dev];
  if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
  return s;
}

namespace {
struct UploadState {   // per host thread and device
  char* stage = nullptr;
  size_t cap = 0, used = 0;
  int depth = 0;             // nested UploadScopes
  bool pending = false;
  int n = 0;                 // IGN_BUILD_PROF counters of the current scope
  size_t bytes = 0, staged = 0;
  double t_copy = 0, t_wait = 0;
  ~UploadState() {   // thread exit (a batch-builder thread): its copies were waited for by its scopes
    if (stage) hipHostFree(stage);
  }
};
UploadState& upload_state() {
  thread_local std::vector<std::unique_ptr<UploadState>> st;   // (owners: the arena is freed once)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if ((int)st.size() <= dev) st.resize(dev + 1);
  if (!st[dev]) st[dev] = std::make_unique<UploadState>();
  return *st[dev];
}
bool env_flag(const char* name, bool dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) != 0 : dflt;
}
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
constexpr size_t kStageMax = (size_t)4 << 20;   // larger copies come from pinned hvec blocks: direct DMA
}  // namespace

hipError_t upload_flush() {
  UploadState& u = upload_state();
  if (!u.pending) return hipSuccess;
  const double t = now_ms();
  const hipError_t e = hipStreamSynchronize(upload_stream());
  u.t_wait += now_ms() - t;
  u.pending = false;
  u.used = 0;
  return e;
}

hipError_t upload_bytes(void* dst, const void* src, size_t bytes) {
  const bool defer = env_flag("IGN_UPLOAD_DEFER", true);   // (read per call: tests switch it)
  UploadState& u = upload_state();
  hipStream_t us = upload_stream();
  u.n++;
  u.bytes += bytes;
  const double t = now_ms();
  hipError_t e;
  if (defer && u.depth > 0 && bytes <= kStageMax) {
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (u.used + need > u.cap) {
      if ((e = upload_flush()) != hipSuccess) return e;   // the arena's copies have landed: reuse it
      if (need > u.cap) {
        if (u.stage) hipHostFree(u.stage);
        u.stage = nullptr;
        u.cap = std::max(need, (size_t)32 << 20);
        if ((e = hipHostMalloc((void**)&u.stage, u.cap, hipHostMallocDefault)) != hipSuccess) {
          u.stage = nullptr;
          u.cap = 0;
          return e;
        }
      }
    }
    char* sp = u.stage + u.used;
    memcpy(sp, src, bytes);
    u.used += need;
    u.staged += bytes;
    u.pending = true;
    e = hipMemcpyAsync(dst, sp, bytes, hipMemcpyHostToDevice, us);
    u.t_copy += now_ms() - t;
    return e;
  }
  e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, us);
  if (e == hipSuccess) {
    u.pending = true;
    e = upload_flush();   // the source may die after the call (and the arena's copies land with it)
  }
  u.t_copy += now_ms() - t;
  return e;
}

UploadScope::UploadScope(const char* w) : what(w), t0(now_ms()) {
  UploadState& u = upload_state();
  if (u.depth++ == 0) {
    u.n = 0;
    u.bytes = u.staged = 0;
    u.t_copy = u.t_wait = 0;
  }
}

UploadScope::~UploadScope() {
  UploadState& u = upload_state();
  // every path out of a builder (errors included) leaves no copy in flight from the arena
  u.pending = true;
  upload_flush();
  if (--u.depth == 0 && env_flag("IGN_BUILD_PROF", false)) {
    int64_t live, idle, maps, unmaps;
    host_cache_stats(&live, &idle, &maps, &unmaps);
    fprintf(stderr,
            "[ign-build] %s: %.2f ms, %d copies, %.1f MB (%.1f MB staged), enqueue %.2f ms, wait %.2f ms; "
            "host blocks live %.0f MB idle %.0f MB, mapped %lld unmapped %lld\n",
            what, now_ms() - t0, u.n, u.bytes / 1e6, u.staged / 1e6, u.t_copy, u.t_wait, live / 1e6, idle / 1e6,
            (long long)maps, (long long)unmaps);
  }
}

int dev_alloc(ign_batch* b, float** out, int64_t n) {
  void* p = nullptr;
  // +256 floats of slack: kernels may read a whole (masked-off) row at index 0 of an empty table
  hipError_t e = pool_alloc(b->pool.get(), &p, (std::max<int64_t>(n, 0) + 256) * sizeof(float), true);
  if (e != hipSuccess) return fail(IGN_ERR_OOM, "device alloc (%lld floats): %s", (long long)n, hipGetErrorString(e));
  b->allocs.push_back(p);
  *out = static_cast<float*>(p);
  return IGN_OK;
}

int act_ok(int a) { return a >= IGN_ACT_LINEAR && a <= IGN_ACT_TANH; }

// Destination processing order: one global stable sort by message count, descending (tiles of
// equal length; the longest sequences start first).  Measured faster than per-graph orders with
// XCD-aware tiles for both the ordered and the sum updates (profiles/r02/seq_experiments).  A
// counting sort (counts are small): O(n), the same order as std::stable_sort.
// f(lo, hi) over [0, n) in contiguous chunks on up to IGN_BUILD_THREADS threads (default 2: a
// training loop already runs several builders), at least min_per items each; the caller's thread
// takes the first chunk
template <class F>
void parallel_ranges(int64_t n, int64_t min_per, F&& f) {
  static const int T = [] {
    const char* v = std::getenv("IGN_BUILD_THREADS");
    return v && *v ? std::max(1, std::atoi(v)) : 2;
  }();
  const int nt = (int)std::min<int64_t>(T, std::max<int64_t>(1, n / std::max<int64_t>(1, min_per)));
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (int t = 1; t < nt; ++t) th.emplace_back([&f, n, nt, t] { f(n * t / nt, n * (t + 1) / nt); });
  f(0, n / nt);
  for (auto& x : th) x.join();
}

void sort_order(hvec<int32_t>& order, const hvec<int64_t>& cnt) {
  const int64_t n = (int64_t)order.size();
  int64_t mx = 0;
  for (int32_t r : order) mx = std::max(mx, cnt[r]);
  if (mx > (int64_t)16 * n + 4096) {
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return cnt[x] > cnt[y]; });
    return;
  }
  hvec<int64_t> start(mx + 2, 0);   // bucket c holds count mx - c (descending)
  for (int32_t r : order) start[mx - cnt[r] + 1]++;
  for (int64_t c = 0; c <= mx; ++c) start[c + 1] += start[c];
  hvec<int32_t> out(n);
  for (int32_t r : order) out[start[mx - cnt[r]]++] = r;
  order.swap(out);
}

// Per-launch algorithmic cost: one GRU application = 2*3H*(DIN+H) + 14H flops.
double gru_flops(int din, int H) { return 2.0 * 3 * H * (din + H) + 14.0 * H; }

}  // namespace ign


int ign::repack(ign_plan* p) {
  for (auto& cp : p->cells) {
    if (!cp.used) continue;
    HIP_TRY(launch_pack_gru(p->d_params + cp.off_k, p->d_params + cp.off_rk, p->d_params + cp.off_b,
                            p->d_packed + cp.pk_w, p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, cp.din, cp.H,
                            p->stream));
    if (cp.pk_ubf >= 0) HIP_TRY(launch_pack_u_bf16(p->d_params + cp.off_rk, p->d_packed + cp.pk_ubf, cp.H, p->stream));
    if (cp.pk_uh >= 0) HIP_TRY(launch_pack_u_f16(p->d_params + cp.off_rk, p->d_packed + cp.pk_uh, cp.H, p->stream));
    if (cp.pk_wh >= 0) HIP_TRY(launch_pack_w_f16(p->d_params + cp.off_k, p->d_packed + cp.pk_wh, cp.din, cp.H, p->stream));
    if (cp.pk_wbf >= 0)
      HIP_TRY(launch_pack_w_bf16(p->d_params + cp.off_k, p->d_packed + cp.pk_wbf, cp.din, cp.H, p->stream));
    if (cp.pk_wt >= 0) HIP_TRY(launch_pack_a(p->d_params + cp.off_k, cp.din, 3 * cp.H, p->d_packed + cp.pk_wt, p->stream));
    if (cp.pk_ut >= 0) HIP_TRY(launch_pack_a(p->d_params + cp.off_rk, cp.H, 3 * cp.H, p->d_packed + cp.pk_ut, p->stream));
    if (cp.pk_uth >= 0) HIP_TRY(launch_pack_ut_f16(p->d_params + cp.off_rk, p->d_packed + cp.pk_uth, cp.H, p->stream));
  }
  for (auto& mp : p->mps)
    if (mp.feature_concat) {
      const CellP& cp = p->cells[mp.cell];
      for (size_t s = 0; s < mp.src.size(); ++s)
        HIP_TRY(launch_pack_gru(p->d_params + cp.off_k + (int64_t)mp.slice_off[s] * 3 * cp.H, nullptr, nullptr,
                                p->d_packed + mp.pk_slice[s], nullptr, nullptr, p->ents[mp.src[s].entity].hidden_dim,
                                cp.H, p->stream));
    }
  for (auto& mp : p->mps)
    for (auto& nn : mp.nn)
      for (size_t l = 0; l < nn.layers.size(); ++l) {
        const DenseP& dp = nn.layers[l];
        if (dp.pk_w >= 0)
          HIP_TRY(launch_pack_dense_pad(p->d_params + dp.off_w, p->d_packed + dp.pk_w, dp.in,
                                        l == 0 ? nn.din_pad : dp.in, dp.out, p->stream));
      }
  if (p->pk_conv >= 0)
    HIP_TRY(launch_pack_dense(p->d_params + p->off_conv, p->d_packed + p->pk_conv, p->conv_F, p->conv_F, p->stream));
  if (p->pk_w12 >= 0)
    HIP_TRY(launch_attn_vectors(p->d_params + p->off_k1, p->d_params + p->off_k2, p->d_params + p->off_att, p->attn_F,
                                p->d_packed + p->pk_w12, p->stream));
  if (p->dense.size() >= 2 && p->dense[1].pk_h >= 0) {
    const DenseP &l1 = p->dense[0], &l2 = p->dense[1];
    HIP_TRY(launch_pack_readout_h16(p->d_params + l1.off_w, l1.use_bias ? p->d_params + l1.off_b : nullptr,
                                    p->d_params + l2.off_w, p->d_packed + l2.pk_h, l1.in, l1.out, l2.out, p->stream));
    if (l2.pk_h32 >= 0)
      HIP_TRY(launch_pack_readout_h32(p->d_params + l1.off_w, l1.use_bias ? p->d_params + l1.off_b : nullptr,
                                      p->d_params + l2.off_w, p->d_packed + l2.pk_h32, l1.in, l1.out, l2.out, p->stream));
  }
  for (auto& dp : p->dense) {
    if (dp.pk_w >= 0) HIP_TRY(launch_pack_dense(p->d_params + dp.off_w, p->d_packed + dp.pk_w, dp.in, dp.out, p->stream));
    if (dp.pk_bf >= 0)   // layer 1 reads its input from memory (natural k), layer 2 chains from registers
      HIP_TRY(launch_pack_dense_bf16(p->d_params + dp.off_w, p->d_packed + dp.pk_bf, dp.in, dp.out, &dp != &p->dense[0],
                                     p->stream));
    if (dp.pk_bfn >= 0)
      HIP_TRY(launch_pack_dense_bf16(p->d_params + dp.off_w, p->d_packed + dp.pk_bfn, dp.in, dp.out, 0, p->stream));
    if (dp.pk_bft >= 0)
      HIP_TRY(launch_pack_dense_bf16_t(p->d_params + dp.off_w, p->d_packed + dp.pk_bft, dp.in, dp.out, p->stream));
    if (dp.pk_hn >= 0)
      HIP_TRY(launch_pack_dense_f16(p->d_params + dp.off_w, p->d_packed + dp.pk_hn, dp.in, dp.out, 0, p->stream));
    if (dp.pk_ht >= 0)
      HIP_TRY(launch_pack_dense_f16(p->d_params + dp.off_w, p->d_packed + dp.pk_ht, dp.out, dp.in, 1, p->stream));
  }
  for (auto& dp : p->dense)
    if (dp.pk_wt >= 0) HIP_TRY(launch_pack_a(p->d_params + dp.off_w, dp.in, dp.out, p->d_packed + dp.pk_wt, p->stream));
  return readout_repack(p);
}

// =============================================================================================
extern "C" {

int ign_abi_version(void) { return IGN_ABI_VERSION; }

const char* ign_last_error(void) { return g_err.c_str(); }

int ign_device_count(int32_t* n) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (n) *n = (e == hipSuccess) ? c : 0;
  return IGN_OK;
}

int ign_plan_create(const ign_plan_desc* d, int32_t device, ign_plan** out) {
  if (!d || !out) return fail(IGN_ERR_INVALID, "null argument");
  *out = nullptr;
  if (d->num_iterations <= 0) return fail(IGN_ERR_INVALID, "num_iterations must be > 0");
  if (d->num_entities <= 0 || d->num_entities > 8) return fail(IGN_ERR_INVALID, "1..8 entities supported");
  std::unique_ptr<ign_plan> p(new ign_plan());
  p->device = device;
  if (const char* v = getenv("IGN_FUSE_PROJ")) p->fuse_proj = atoi(v) != 0;
  if (const char* v = getenv("IGN_SEQ_VARIANT")) {   // 6 (default), 4 or 2; anything else: 6
    const int sv = atoi(v);
    p->seq_variant = sv == 2 || sv == 4 ? sv : 6;
  }
  if (const char* v = getenv("IGN_HIP_GRAPH")) p->use_graph = atoi(v) != 0;
  if (const char* v = getenv("IGN_SUM_VARIANT")) p->sum_variant = atoi(v) == 7 || atoi(v) == 8 ? atoi(v) : 3;
  if (const char* v = getenv("IGN_SUM_WINDOW")) p->sum_window = atoi(v);
  if (const char* v = getenv("IGN_RESIDENT")) {   // 0 off; 1 default; 2 also force the global-path form
    p->resident = atoi(v) != 0;
    p->resident_path_global = atoi(v) == 2;
  }
  if (const char* v = getenv("IGN_RESIDENT_PG")) p->resident_pg = atoi(v) != 0;
  if (const char* v = getenv("IGN_RESIDENT_TRAIN")) p->resident_train = atoi(v) != 0;
  if (const char* v = getenv("IGN_RES_LPT")) p->res_lpt = atoi(v) != 0;
  if (const char* v = getenv("IGN_RES_GROUP")) p->res_group = std::max(0, atoi(v));
  if (const char* v = getenv("IGN_RESIDENT_SAVE_TABLE")) p->resident_save_table = atoi(v) != 0;
  if (const char* v = getenv("IGN_BWD_FUSE")) p->bwd_fuse = atoi(v) != 0;
  if (const char* v = getenv("IGN_SUM_BWD_FUSE")) p->sum_bwd_fuse = atoi(v) != 0;
  if (const char* v = getenv("IGN_TRAIN_DENSE_BF")) p->train_dense_bf = atoi(v) != 0;
  if (const char* v = getenv("IGN_TRAIN_DENSE_H16")) p->train_dense_h16 = atoi(v) != 0;
  if (const char* v = getenv("IGN_TSGEMM_BF")) p->tsgemm_bf = atoi(v) != 0;
  if (const char* v = getenv("IGN_FUSE_OUTER_BWD")) p->fuse_outer_bwd = atoi(v) != 0;
  if (const char* v = getenv("IGN_TRAIN_FUSED_READOUT")) p->train_fused_readout = atoi(v) != 0;
  if (const char* v = getenv("IGN_BWD_BF")) p->bwd_bf = atoi(v) != 0;
  if (const char* v = getenv("IGN_TRAIN_SEQ_H16")) p->train_seq_h16 = atoi(v) != 0;
  if (const char* v = getenv("IGN_READOUT_VARIANT")) {   // 4 (default), 5, 2 or 1; anything else: 4
    const int rv = atoi(v);
    p->readout_variant = rv == 1 || rv == 2 || rv == 5 ? rv : 4;
  }
  p->T = d->num_iterations;
  p->ents.assign(d->entities, d->entities + d->num_entities);
  for (size_t e = 0; e < p->ents.size(); ++e) {
    const auto& en = p->ents[e];
    if (en.hidden_dim <= 0) return fail(IGN_ERR_INVALID, "entity %zu: hidden_state_dimension must be > 0", e);
    if (en.feature_total > en.hidden_dim)   // AUX:155-159: zeros(H - total) needs total <= H
      return fail(IGN_ERR_INVALID, "entity %zu: total feature size %d exceeds hidden_state_dimension %d", e,
                  en.feature_total, en.hidden_dim);
  }
  p->n_adj = d->num_adjacencies;
  p->n_il = d->num_interleave;
  for (int c = 0; c < d->num_cells; ++c) {
    CellP cp;
    cp.din = d->cells[c].input_dim;
    cp.H = d->cells[c].units;
    p->cells.push_back(cp);
  }
  for (int m = 0; m < d->num_mps; ++m) {
    const ign_mp_desc& md = d->mps[m];
    MPP mp;
    mp.dst = md.dst_entity;
    mp.aggr = md.aggregation;
    mp.concat_axis = md.concat_axis;
    mp.cell = md.cell;
    if (mp.dst < 0 || mp.dst >= d->num_entities) return fail(IGN_ERR_INVALID, "mp %d: bad destination", m);
    if (md.num_sources <= 0) return fail(IGN_ERR_INVALID, "mp %d: no source entities", m);
    if (md.num_sources > IGN_MAX_SLOTS)
      return fail(IGN_ERR_UNSUPPORTED, "mp %d: more than %d source entities", m, IGN_MAX_SLOTS);
    mp.src.assign(md.sources, md.sources + md.num_sources);
    switch (mp.aggr) {
      case IGN_AGGR_SUM: mp.sorted = false; break;
      case IGN_AGGR_ORDERED: mp.sorted = true; break;
      case IGN_AGGR_INTERLEAVE:
        mp.sorted = true;
        if (md.num_sources != 2)  // tf.stack of the index lists (GM:518) needs exactly two sources
          return fail(IGN_ERR_UNSUPPORTED, "mp %d: interleave aggregation supports exactly 2 sources (GM:518)", m);
        break;
      case IGN_AGGR_CONCAT:
        if (mp.concat_axis != 1 && mp.concat_axis != 2)
          return fail(IGN_ERR_INVALID, "mp %d: concat_axis must be 1 or 2", m);
        mp.sorted = true;
        mp.feature_concat = mp.concat_axis == 2;
        break;
      case IGN_AGGR_ATTENTION:
      case IGN_AGGR_CONVOLUTION:
        mp.sorted = false;
        mp.act = md.activation;
        if (mp.aggr == IGN_AGGR_CONVOLUTION && !act_ok(mp.act))
          return fail(IGN_ERR_UNSUPPORTED, "mp %d: convolution activation %d", m, mp.act);
        break;
      default:
        return fail(IGN_ERR_UNSUPPORTED, "mp %d: aggregation %d is not lowered", m, mp.aggr);
    }
    int din = -1;
    for (auto& s : mp.src) {
      if (s.entity < 0 || s.entity >= d->num_entities) return fail(IGN_ERR_INVALID, "mp %d: bad source entity", m);
      if (s.adjacency < 0 || s.adjacency >= p->n_adj) return fail(IGN_ERR_INVALID, "mp %d: bad adjacency slot", m);
      if (mp.aggr == IGN_AGGR_INTERLEAVE && (s.interleave < 0 || s.interleave >= p->n_il))
        return fail(IGN_ERR_INVALID, "mp %d: interleave slot missing", m);
      int dm = p->ents[s.entity].hidden_dim;   // direct_assignation: message = source state
      MsgNN nn;
      if (s.msg_num_layers > 0) {               // message-creation network (GM:440-475)
        nn.param_dim = s.msg_param_dim;
        for (int q = 0; q < s.msg_num_inputs; ++q) {
          const int kind = s.msg_inputs[q];
          nn.inputs.push_back(kind);
          int w = 0;
          if (kind == IGN_MSG_HS_SOURCE) w = p->ents[s.entity].hidden_dim;
          else if (kind == IGN_MSG_HS_DEST) w = p->ents[mp.dst].hidden_dim;
          else if (kind == IGN_MSG_EDGE_PARAMS) w = s.msg_param_dim;
          else return fail(IGN_ERR_UNSUPPORTED, "mp %d: message input %d is not lowered", m, kind);
          if (w <= 0) return fail(IGN_ERR_INVALID, "mp %d: message input %d has no width", m, kind);
          if (q >= 4) return fail(IGN_ERR_UNSUPPORTED, "mp %d: more than 4 message inputs", m);
          nn.widths.push_back(w);
          nn.din += w;
        }
        if (nn.din <= 0) return fail(IGN_ERR_INVALID, "mp %d: empty message-network input", m);
        nn.din_pad = (nn.din + 15) / 16 * 16;
        int in = nn.din;
        for (int l = 0; l < s.msg_num_layers; ++l) {
          DenseP dp;
          dp.in = in;
          dp.out = s.msg_layers[l].units;
          dp.act = s.msg_layers[l].activation;
          dp.use_bias = s.msg_layers[l].use_bias;
          dp.l2 = s.msg_layers[l].l2;   // kernel_regularizer: part of model.losses (AUX:833-834)
          if (dp.out <= 0) return fail(IGN_ERR_INVALID, "mp %d: message layer %d units", m, l);
          if (!act_ok(dp.act)) return fail(IGN_ERR_UNSUPPORTED, "mp %d: message layer activation %d", m, dp.act);
          nn.layers.push_back(dp);
          in = dp.out;
        }
        dm = nn.dout();
      }
      mp.nn.push_back(nn);
      if (mp.feature_concat) {                 // axis 2: the step input is the sources' concatenation
        mp.slice_off.push_back(din < 0 ? 0 : din);
        din = (din < 0 ? 0 : din) + dm;
        continue;
      }
      if (din >= 0 && dm != din)
        return fail(IGN_ERR_INVALID, "mp %d: sources have different message dimensions (%d vs %d)", m, din, dm);
      din = dm;
    }
    mp.din = din;
    if (mp.cell < 0 || mp.cell >= (int)p->cells.size()) return fail(IGN_ERR_INVALID, "mp %d: bad cell index", m);
    CellP& cp = p->cells[mp.cell];
    if (cp.H != p->ents[mp.dst].hidden_dim)
      return fail(IGN_ERR_INVALID, "mp %d: cell units %d != destination hidden dim %d", m, cp.H, p->ents[mp.dst].hidden_dim);
    if (cp.din != din)
      return fail(IGN_ERR_INVALID, "mp %d: cell input_dim %d != message dim %d", m, cp.din, din);
    if (mp.feature_concat) {   // x.W is hoisted per source slice: the shapes that matter are (slice, H)
      for (auto& s : mp.src)
        if (!gru_shape_supported(p->ents[s.entity].hidden_dim, cp.H))
          return fail(IGN_ERR_UNSUPPORTED, "mp %d: concat slice (input %d, units %d) not instantiated", m,
                      p->ents[s.entity].hidden_dim, cp.H);
    } else if (!gru_shape_supported(din, cp.H)) {
      return fail(IGN_ERR_UNSUPPORTED, "mp %d: GRU shape (input %d, units %d) not instantiated (16/32, 64/64)", m,
                  din, cp.H);
    }
    if (mp.aggr == IGN_AGGR_ATTENTION || mp.aggr == IGN_AGGR_CONVOLUTION) {
      const int F = p->ents[mp.dst].hidden_dim;
      // AUX:311-319 / GM:293-298: the messages and the destination states must have one width
      if (din != F)
        return fail(IGN_ERR_INVALID, "mp %d: %s needs message dim %d == destination dim %d", m,
                    mp.aggr == IGN_AGGR_ATTENTION ? "attention" : "convolution", din, F);
      if (F != 16 && F != 32)
        return fail(IGN_ERR_UNSUPPORTED, "mp %d: attention / convolution lowered for 16 or 32 units", m);
      int& pf = mp.aggr == IGN_AGGR_ATTENTION ? p->attn_F : p->conv_F;
      if (pf && pf != F)
        return fail(IGN_ERR_INVALID, "mp %d: the shared %s weights have width %d, this MP needs %d (GM:288-300)", m,
                    mp.aggr == IGN_AGGR_ATTENTION ? "attention" : "convolution", pf, F);
      pf = F;
    }
    cp.used = true;
    p->mps.push_back(mp);
  }
  // readout program and predict (GM:605-629)
  if (int rc = readout_plan(p.get(), d)) return rc;

  // parameter layout (256-B aligned tensors)
  auto align = [](int64_t x) { return (x + 63) & ~int64_t(63); };
  int64_t off = 0;
  for (size_t c = 0; c < p->cells.size(); ++c) {
    CellP& cp = p->cells[c];
    int g3 = 3 * cp.H;
    cp.off_k = off; p->tensors.push_back({0, (int)c, off, cp.din, g3}); off = align(off + (int64_t)cp.din * g3);
    cp.off_rk = off; p->tensors.push_back({1, (int)c, off, cp.H, g3}); off = align(off + (int64_t)cp.H * g3);
    cp.off_b = off; p->tensors.push_back({2, (int)c, off, 2, g3}); off = align(off + 2LL * g3);
  }
  for (size_t mi = 0; mi < p->mps.size(); ++mi)
    for (size_t s = 0; s < p->mps[mi].nn.size(); ++s)
      for (auto& dp : p->mps[mi].nn[s].layers) {
        const int owner = (int)(mi * IGN_MAX_SLOTS + s);
        dp.off_w = off; p->tensors.push_back({9, owner, off, dp.in, dp.out}); off = align(off + (int64_t)dp.in * dp.out);
        if (dp.use_bias) { dp.off_b = off; p->tensors.push_back({10, owner, off, 1, dp.out}); off = align(off + dp.out); }
      }
  if (p->conv_F) {
    const int F = p->conv_F;
    p->off_conv = off; p->tensors.push_back({5, -1, off, F, F}); off = align(off + (int64_t)F * F);
  }
  if (p->attn_F) {
    const int F = p->attn_F;
    p->off_k1 = off; p->tensors.push_back({6, -1, off, F, F}); off = align(off + (int64_t)F * F);
    p->off_k2 = off; p->tensors.push_back({7, -1, off, F, F}); off = align(off + (int64_t)F * F);
    p->off_att = off; p->tensors.push_back({8, -1, off, 2 * F, 1}); off = align(off + 2LL * F);
  }
  off = readout_layout(p.get(), off);
  for (size_t l = 0; l < p->dense.size(); ++l) {
    DenseP& dp = p->dense[l];
    dp.off_w = off; p->tensors.push_back({3, (int)l, off, dp.in, dp.out}); off = align(off + (int64_t)dp.in * dp.out);
    dp.off_b = off; p->tensors.push_back({4, (int)l, off, 1, dp.out}); off = align(off + dp.out);
  }
  p->n_params = off;
  int64_t pk = 0;
  for (auto& cp : p->cells) {
    if (!cp.used) continue;
    cp.pk_w = pk; pk = align(pk + 3LL * cp.din * cp.H);
    cp.pk_u = pk; pk = align(pk + 3LL * cp.H * cp.H);
    cp.pk_b = pk; pk = align(pk + 4LL * cp.H);
    if (pack_u_bf16_floats(cp.H)) { cp.pk_ubf = pk; pk = align(pk + pack_u_bf16_floats(cp.H)); }
    if (pack_u_f16_floats(cp.H)) { cp.pk_uh = pk; pk = align(pk + pack_u_f16_floats(cp.H)); }
    if (cp.din == 64 && cp.H == 64) { cp.pk_wh = pk; pk = align(pk + pack_w_f16_floats(cp.din, cp.H)); }
    if ((cp.din == 64 && cp.H == 64) || (cp.din == 32 && cp.H == 32)) { cp.pk_wbf = pk; pk = align(pk + pack_w_bf16_floats(cp.din, cp.H)); }
  }
  for (size_t l = 0; l < p->dense.size(); ++l) {
    DenseP& dp = p->dense[l];
    if ((p->fused_readout && l < 2) || dense_fwd_supported(dp.in, dp.out)) {
      dp.pk_w = pk;
      pk = align(pk + (int64_t)dp.in * dp.out);
    }
    if (p->fused_readout && l < 2 && dp.in % 32 == 0 && dp.out % 16 == 0 &&
        readout_bf_supported(p->dense[0].in, p->dense[0].out, p->dense[1].out, p->dense[0].act, p->dense[1].act)) {
      dp.pk_bf = pk;
      pk = align(pk + 3LL * dp.in * dp.out / 2);
      if (l == 1) {
        dp.pk_h = pk; pk = align(pk + (int64_t)dp.in * dp.out + 64 + (int64_t)p->dense[0].in * dp.in + 64);
        if (p->readout_variant == 5)   // (otherwise neither packed after each optimizer step nor allocated)
          dp.pk_h32 = pk, pk = align(pk + (int64_t)dp.in * dp.out + 64 + (int64_t)p->dense[0].in * dp.in + 64);
      }
    }
    if (dense_bf_supported(dp.in, dp.out)) {
      dp.pk_bfn = pk;
      pk = align(pk + 3LL * dp.in * dp.out / 2);
      dp.pk_hn = pk;
      pk = align(pk + (int64_t)dp.in * dp.out + 64);
    }
    if (dense_bf_supported(dp.out, dp.in)) {
      dp.pk_bft = pk;
      pk = align(pk + 3LL * dp.in * dp.out / 2);
      dp.pk_ht = pk;
      pk = align(pk + (int64_t)dp.in * dp.out + 64);
    }
  }
  // backward fragments (training): W^T / U^T per cell, W^T per Dense layer where the MFMA
  // row GEMM is instantiated
  for (auto& cp : p->cells) {
    if (!cp.used || !bwd_shape_supported(cp.H, cp.H)) continue;   // U^T: the recurrent backward
    cp.pk_ut = pk; pk = align(pk + 3LL * cp.H * cp.H);
    if (pack_ut_f16_floats(cp.H)) { cp.pk_uth = pk; pk = align(pk + pack_ut_f16_floats(cp.H)); }
    if (!bwd_shape_supported(cp.din, cp.H)) continue;            // W^T (an axis-2 concat cell goes generic)
    cp.pk_wt = pk; pk = align(pk + 3LL * cp.din * cp.H);
  }
  for (auto& dp : p->dense) {
    if (!row_gemm_supported(dp.out, dp.in)) continue;
    dp.pk_wt = pk; pk = align(pk + (int64_t)dp.in * dp.out);
  }
  for (auto& mp : p->mps)
    for (auto& nn : mp.nn)
      for (size_t l = 0; l < nn.layers.size(); ++l) {
        DenseP& dp = nn.layers[l];
        const int kin = l == 0 ? nn.din_pad : dp.in;
        if (dense_fwd_supported(kin, dp.out)) { dp.pk_w = pk; pk = align(pk + (int64_t)kin * dp.out); }
      }
  for (auto& mp : p->mps)
    if (mp.feature_concat)
      for (auto& s : mp.src) {
        mp.pk_slice.push_back(pk);
        pk = align(pk + 3LL * p->ents[s.entity].hidden_dim * p->cells[mp.cell].H);
      }
  if (p->conv_F) { p->pk_conv = pk; pk = align(pk + (int64_t)p->conv_F * p->conv_F); }
  if (p->attn_F) { p->pk_w12 = pk; pk = align(pk + 2LL * p->attn_F); }
  pk = readout_packed(p.get(), pk);
  p->n_packed = pk;

  // Device resources are allocated on first use (ensure_device), so plan validation and the
  // parameter layout are available without a GPU.
  *out = p.release();
  return IGN_OK;
}

void ign_plan_destroy(ign_plan* p) {
  if (!p) return;
  if (!p->d_params && !p->stream) {
    delete p;
    return;
  }
  hipSetDevice(p->device);
  if (p->stream) hipStreamSynchronize(p->stream);
  for (auto e : p->ev) hipEventDestroy(e);
  if (p->d_params) hipFree(p->d_params);
  if (p->d_packed) hipFree(p->d_packed);
  if (p->d_red) hipFree(p->d_red);
  if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
  delete p;
}

int ign_plan_num_params(const ign_plan* p, int64_t* n) {
  if (!p || !n) return fail(IGN_ERR_INVALID, "null argument");
  *n = p->n_params;
  return IGN_OK;
}

int ign_plan_num_param_tensors(const ign_plan* p, int32_t* n) {
  if (!p || !n) return fail(IGN_ERR_INVALID, "null argument");
  *n = (int32_t)p->tensors.size();
  return IGN_OK;
}

int ign_plan_param_tensor(const ign_plan* p, int32_t i, int32_t* kind, int32_t* owner, int64_t* offset,
                          int32_t* rows, int32_t* cols) {
  if (!p || i < 0 || i >= (int)p->tensors.size()) return fail(IGN_ERR_INVALID, "tensor index out of range");
  const Tensor& t = p->tensors[i];
  if (kind) *kind = t.kind;
  if (owner) *owner = t.owner;
  if (offset) *offset = t.offset;
  if (rows) *rows = t.rows;
  if (cols) *cols = t.cols;
  return IGN_OK;
}

int ign_plan_set_params(ign_plan* p, const float* params, int32_t on_device) {
  if (!p || !params) return fail(IGN_ERR_INVALID, "null argument");
  int rc = ensure_device(p);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(p->d_params, params, p->n_params * sizeof(float),
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, p->stream));
  if ((rc = repack(p))) return rc;
  HIP_TRY(hipStreamSynchronize(p->stream));
  p->params_set = true;
  return IGN_OK;
}

namespace {
// timed launches record event pairs into a ring on the plan; they are resolved lazily
constexpr int kMaxPendingEvents = 1 << 14;
int flush_timing(ign_plan* p);
void drop_timing(ign_plan* p);
}  // namespace

int ign_plan_set_timing(ign_plan* p, int32_t enabled) {
  if (!p) return fail(IGN_ERR_INVALID, "null plan");
  drop_timing(p);
  p->timing = enabled != 0;
  p->stats = ign_stats_t{};
  return IGN_OK;
}

int ign_plan_set_timing_kinds(ign_plan* p, uint32_t kinds) {
  if (!p) return fail(IGN_ERR_INVALID, "null plan");
  drop_timing(p);
  p->timing_kinds = kinds;
  p->stats = ign_stats_t{};
  return IGN_OK;
}

int ign_plan_set_stream(ign_plan* p, void* s) {
  if (!p) return fail(IGN_ERR_INVALID, "null plan");
  int rc = ensure_device(p);
  if (rc) return rc;
  if ((rc = flush_timing(p))) return rc;   // pending event pairs were recorded on the old stream
  // Pooled blocks of destroyed batches carry a fence recorded on the plan's stream at destroy time;
  // from here on fences go to the new stream, so work still queued on the old one (own or external)
  // must finish before a block it reads can be handed out again.
  if (p->stream && p->stream != static_cast<hipStream_t>(s)) HIP_TRY(hipStreamSynchronize(p->stream));
  if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
  p->own_stream = false;
  p->external_stream = true;
  p->stream = static_cast<hipStream_t>(s);
  return IGN_OK;
}

// ---------------------------------------------------------------------------------------------
// The graph-resident forward (resident.hip): one ordered MP into the "path" entity from S <= 2
// source entities (plain, one message per position) and, for each source entity, one sum MP from
// the paths back to it, every MP at H = DIN = 32 on the default split kernels (RouteNet: S = 1;
// Q-size: links and nodes interleaved, S = 2), on graphs whose states and projected table fit one
// workgroup's LDS.  Otherwise the batched path.
struct ResShape {
  int path = -1, n_src = 0;
  int src_ent[kResidentMaxSrc] = {-1, -1};
  int sum_mp[kResidentMaxSrc] = {-1, -1};
};

static bool resident_plan_shape(const ign_plan* p, ResShape* sh) {
  // the windowed sum (IGN_SUM_WINDOW=1) adds in another order: not restated here
  if (!p->resident || !p->fuse_proj || p->seq_variant != 6 || p->sum_variant < 7 || p->sum_window == 1) return false;
  const int n = (int)p->mps.size();
  if (n < 2 || n > kResidentMaxSrc + 1 || (int)p->ents.size() != n) return false;
  const MPP& a = p->mps[0];
  const int S = (int)a.src.size();
  if (!a.sorted || S + 1 != n || a.feature_concat || a.din != 32) return false;
  const CellP& ca = p->cells[a.cell];
  if (ca.H != 32 || ca.pk_uh < 0 || ca.pk_wbf < 0 || ca.pk_w < 0) return false;
  sh->path = a.dst;
  sh->n_src = S;
  for (int s = 0; s < S; ++s) {
    const int e = a.src[s].entity;
    if (e == a.dst || !a.nn[s].layers.empty()) return false;
    for (int t = 0; t < s; ++t)
      if (sh->src_ent[t] == e) return false;
    sh->src_ent[s] = e;
  }
  // MPs 1 .. S: one sum MP path -> each source entity, in any order (they read only the paths)
  for (int m = 1; m < n; ++m) {
    const MPP& q = p->mps[m];
    int s = -1;
    for (int t = 0; t < S; ++t)
      if (sh->src_ent[t] == q.dst) s = t;
    if (s < 0 || sh->sum_mp[s] >= 0) return false;
    if (q.sorted || q.aggr != IGN_AGGR_SUM || q.src.size() != 1 || q.src[0].entity != a.dst || q.feature_concat ||
        !q.nn[0].layers.empty() || q.din != 32)
      return false;
    const CellP& cq = p->cells[q.cell];
    if (cq.H != 32 || cq.pk_wbf < 0 || cq.pk_ubf < 0) return false;
    sh->sum_mp[s] = m;
  }
  for (int e = 0; e < n; ++e)
    if (p->ents[e].feature_total > 32 || p->ents[e].hidden_dim != 32) return false;
  return true;
}

// dynamic LDS of one graph in a form: union-row states and projected table always; the sum MPs' CSR
// rows unless CL is off; the path states and step codes in the all-LDS form
static size_t resident_lds_bytes(int64_t paths, int64_t urows, int64_t msgs, int64_t codes, int form) {
  const size_t order = (size_t)((urows + 1) & ~int64_t(1)) * sizeof(uint16_t);   // the row order, padded
  size_t b = (size_t)(urows * kResidentStateStride + (urows + 1) * kResidentTableStride) * sizeof(float) +
             (size_t)(urows + 1) * sizeof(int32_t) + order;
  if (form != IGN_RES_PATH_CSR_GLOBAL) b += (size_t)msgs * sizeof(uint16_t);
  if (form == IGN_RES_ALL_LDS) b += (size_t)paths * kResidentStateStride * sizeof(float) + (size_t)codes * sizeof(uint16_t);
  return b;
}

// a sum MP's destinations with at least this many messages take the segmented sum (sum_seg_kernel,
// one wave per destination); the others the lane walk of the GRU-step kernel (IGN_SUM_WINDOW=2: every
// destination segmented).  Per destination, so a graph's rows take the same order alone and in any batch.
// IGN_SUM_WINDOW=0, the lane walk's A/B switch, refuses a batch with a destination of >= 64 messages
// (ign_batch_create): a float32 chain that long leaves the fp32 class -- Q-size synth50's nodes as
// lane walks landed at 4.3x IEEE float32's error (all of them) and 1.8x (those below 128), DESIGN.md §4
constexpr int64_t kSegMinMessages = 64;
static int64_t seg_min_messages(const ign_plan* p) { return p->sum_window == 2 ? 0 : kSegMinMessages; }

// per-graph tables of the resident forward, K graphs per workgroup; leaves b->resident false where it
// does not apply
static int resident_batch_k(ign_plan* p, ign_batch* b, int K) {
  ResShape sh;
  if (!resident_plan_shape(p, &sh)) return IGN_OK;
  const int path = sh.path, S = sh.n_src;
  const MPB& ma = b->mp[0];
  if (b->halo[path] || ma.n_multi || (int)ma.src_off.size() != S) return IGN_OK;
  for (int s = 0; s < S; ++s)
    if (b->halo[sh.src_ent[s]]) return IGN_OK;
  // a workgroup's "graph" is a group of K consecutive graphs of the batch (round 6, IGN_RES_GROUP):
  // their disjoint union is one graph to the kernel (concatenated local rows, one tile counter, one
  // set of union-row tiles), so small graphs fill the 16 waves -- GEANT2's 35 path tiles and 5
  // union-row tiles per graph leave most waves idle in phase A's tail and in phase B.  Every row is
  // computed as before (tiles of paths sorted by length across the group: the scale caveat above)
  const int G = (b->G + K - 1) / K;
  std::vector<int64_t> po_g(G + 1), so_g[kResidentMaxSrc];
  for (int k = 0; k <= G; ++k) po_g[k] = b->row_off[path][std::min(k * K, b->G)];
  for (int s = 0; s < S; ++s) {
    so_g[s].resize(G + 1);
    for (int k = 0; k <= G; ++k) so_g[s][k] = b->row_off[sh.src_ent[s]][std::min(k * K, b->G)];
  }
  const auto& po = po_g;
  const std::vector<int64_t>* so[kResidentMaxSrc] = {&so_g[0], S > 1 ? &so_g[1] : nullptr};
  auto Ls = [&](int s, int g) -> int64_t { return s < S ? (*so[s])[g + 1] - (*so[s])[g] : 0; };
  // union rows: per graph, source entity 0's rows, then entity 1's
  std::vector<int64_t> uo(G + 1, 0);
  for (int g = 0; g < G; ++g) {
    uo[g + 1] = uo[g] + Ls(0, g) + Ls(1, g);
    if (po[g + 1] - po[g] > 65535 || uo[g + 1] - uo[g] > 65535) return IGN_OK;   // local rows are 16-bit
    if ((Ls(0, g) + 15) / 16 + (Ls(1, g) + 15) / 16 > kResidentMaxTiles) return IGN_OK;   // B2/B3: two tiles per wave
  }
  // the graph of every row (rows are graph-contiguous)
  auto graph_of = [&](const std::vector<int64_t>& off, int64_t r) {
    return (int)(std::upper_bound(off.begin(), off.end(), r) - off.begin()) - 1;
  };
  auto urow = [&](int s, int g, int64_t row) { return uo[g] + (s ? Ls(0, g) : 0) + (row - (*so[s])[g]); };
  // the sum MPs: each graph's CSR by local union row, its messages in the MP's order (local path rows)
  hvec<int32_t> lmsg_ptr((size_t)(uo[G] + G), 0), lmsg_off(G + 1, 0);
  std::vector<int64_t> nmsg(G, 0);
  for (int s = 0; s < S; ++s) {
    const MPB& ms = b->mp[sh.sum_mp[s]];
    for (int64_t q = 0; q < (int64_t)ms.h_order.size(); ++q) {
      const int64_t row = ms.h_order[q];
      const int g = graph_of(*so[s], row);
      const int32_t cnt = ms.h_msg_ptr[q + 1] - ms.h_msg_ptr[q];
      lmsg_ptr[urow(s, g, row) + g + 1] = cnt;   // counts, prefix-summed below
      nmsg[g] += cnt;
    }
  }
  const int64_t seg_min = seg_min_messages(p);
  hvec<uint16_t> lorder(std::max<int64_t>(uo[G], 1));
  hvec<int32_t> lnseg(G, 0);
  int64_t seg_rows = 0;
  for (int g = 0; g < G; ++g) {
    lmsg_off[g + 1] = lmsg_off[g] + (int32_t)nmsg[g];
    int32_t* cp = lmsg_ptr.data() + uo[g] + g;
    const int64_t U = uo[g + 1] - uo[g];
    // its local rows by message count, descending (stable): the rows of >= seg_min messages first
    // (the segmented sums), then the lane walks, long chains first
    std::vector<int32_t> ord(U);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return cp[x + 1] > cp[y + 1]; });
    for (int64_t r = 0; r < U; ++r) {
      lorder[uo[g] + r] = (uint16_t)ord[r];
      if (cp[ord[r] + 1] >= seg_min) lnseg[g]++;
    }
    seg_rows += lnseg[g];
    for (int64_t r = 0; r < U; ++r) cp[r + 1] += cp[r];
  }
  hvec<uint16_t> lmsg_src(std::max<int32_t>(lmsg_off[G], 1));
  for (int s = 0; s < S; ++s) {
    const MPB& ms = b->mp[sh.sum_mp[s]];
    for (int64_t q = 0; q < (int64_t)ms.h_order.size(); ++q) {
      const int64_t row = ms.h_order[q];
      const int g = graph_of(*so[s], row);
      int32_t pos = lmsg_off[g] + lmsg_ptr[urow(s, g, row) + g];
      for (int32_t m = ms.h_msg_ptr[q]; m < ms.h_msg_ptr[q + 1]; ++m) {
        const int64_t pr = (int64_t)(ms.h_msg_src[m] & IGN_ROW_MASK) - po[g];
        if ((ms.h_msg_src[m] >> IGN_SLOT_SHIFT) != 0 || pr < 0 || pr >= po[g + 1] - po[g]) return IGN_OK;
        lmsg_src[pos++] = (uint16_t)pr;
      }
    }
  }
  // ordered MP: each graph's positions in the batch's length-sorted order (stable, so still sorted
  // by length, descending), padded to whole tiles; their step codes as local union rows (U_g: the
  // hole), then max_len + 8 hole codes (the tile loop reads codes past a row's end)
  // (positions by graph: a counting sort keyed by a row -> graph table, the batch order kept)
  const int64_t ND = (int64_t)ma.h_order.size();
  hvec<int32_t> pstart(G + 1, 0), plist(std::max<int64_t>(ND, 1));
  {
    hvec<int32_t> gid(std::max<int64_t>(po[G], 1));
    for (int g = 0; g < G; ++g)
      for (int64_t r = po[g]; r < po[g + 1]; ++r) gid[r] = g;
    for (int64_t i = 0; i < ND; ++i) pstart[gid[ma.h_order[i]] + 1]++;
    for (int g = 0; g < G; ++g) pstart[g + 1] += pstart[g];
    hvec<int32_t> fill(pstart.begin(), pstart.end() - 1);
    for (int64_t i = 0; i < ND; ++i) plist[fill[gid[ma.h_order[i]]]++] = (int32_t)i;
  }
  // two passes over the graphs, the second on IGN_BUILD_THREADS threads (the tables are ~10^7
  // entries for 512 synth50 graphs, ~20 ms on one builder thread): each graph's sizes, their
  // prefix sums, then every graph fills its own ranges
  std::vector<int64_t> npad(G), ncode(G), maxl_g(G, 0);
  hvec<int32_t> ptile_off(G + 1, 0), lcode_off(G + 1, 0);
  double tile_steps = 0;
  for (int g = 0; g < G; ++g) {
    const int64_t n = pstart[g + 1] - pstart[g];
    npad[g] = (n + 15) / 16 * 16;
    int64_t codes = 0, maxl = 0;
    for (int64_t k = pstart[g]; k < pstart[g + 1]; ++k) {
      const int32_t len = ma.h_len[plist[k]];
      codes += len;
      maxl = std::max<int64_t>(maxl, len);
    }
    for (int64_t k = pstart[g]; k < pstart[g + 1]; k += 16) tile_steps += ma.h_len[plist[k]];   // a tile's first row is its longest
    maxl_g[g] = maxl;
    ncode[g] = codes + maxl + 8;
    ptile_off[g + 1] = ptile_off[g] + (int32_t)npad[g];
    if ((int64_t)lcode_off[g] + ncode[g] >= INT32_MAX) return IGN_OK;
    lcode_off[g + 1] = lcode_off[g] + (int32_t)ncode[g];
  }
  hvec<int32_t> hdr((size_t)4 * ptile_off[G]), hsb((size_t)ptile_off[G]);
  hvec<uint16_t> lcode((size_t)lcode_off[G]);
  std::atomic<bool> foreign{false};   // a code of another graph's row or a multi-message row: not resident
  parallel_ranges(G, 16, [&](int64_t g0, int64_t g1) {
    for (int64_t g = g0; g < g1 && !foreign.load(std::memory_order_relaxed); ++g) {
      const int64_t U = uo[g + 1] - uo[g];
      int32_t* h = hdr.data() + (size_t)4 * ptile_off[g];
      int32_t* hs = hsb.data() + ptile_off[g];
      uint16_t* lc = lcode.data() + lcode_off[g];
      int32_t c = 0;   // the graph's next local code
      for (int64_t k = pstart[g]; k < pstart[g + 1]; ++k) {
        const int64_t i = plist[k];
        const int32_t len = ma.h_len[i], sp = ma.h_step_ptr[i];
        *h++ = (int32_t)(ma.h_order[i] - po[g]);
        *h++ = len;
        *hs++ = sp + (int32_t)i;   // the training forward's hs_save rows of position i
        *h++ = c;
        const int32_t c_first = c;
        for (int32_t t = 0; t < len; ++t) {
          const uint32_t cd = ma.h_step_code[sp + t];
          uint16_t code = (uint16_t)U;   // the zero row: a hole
          if (cd < (uint32_t)ma.zero_row) {
            const int s = S > 1 && (int64_t)cd >= ma.src_off[1] ? 1 : 0;
            const int64_t lr = (int64_t)cd - ma.src_off[s] - (*so[s])[g];
            if (lr < 0 || lr >= Ls(s, (int)g)) { foreign = true; return; }
            code = (uint16_t)((s ? Ls(0, (int)g) : 0) + lr);
          } else if (cd != (uint32_t)ma.zero_row) {
            foreign = true;   // a multi-message row (n_multi == 0: unreachable)
            return;
          }
          lc[c++] = code;
        }
        *h++ = len > 0 ? lc[c_first] : (int32_t)U;
      }
      const int32_t pad = c;
      for (int64_t q = 0; q < maxl_g[g] + 8; ++q) lc[c++] = (uint16_t)U;
      for (int64_t k = pstart[g + 1] - pstart[g]; k < npad[g]; ++k) {   // padding: row -1, length 0, hole codes, hs_save's pad row (unwritten)
        *hs++ = (int32_t)(ma.n_steps + ND);
        *h++ = -1;
        *h++ = 0;
        *h++ = pad;
        *h++ = (int32_t)U;
      }
    }
  });
  if (foreign) return IGN_OK;
  size_t lds[3] = {0, 0, 0};
  for (int g = 0; g < G; ++g)
    for (int f = 0; f < 3; ++f)
      lds[f] = std::max(lds[f], resident_lds_bytes(po[g + 1] - po[g], uo[g + 1] - uo[g], nmsg[g], ncode[g], f));
  // the workgroups' graphs, longest first (round 6): a launch of more graphs than CUs -- or the second
  // of two sub-batch launches, whose workgroups take the CUs the first one frees -- is a list
  // schedule in workgroup order, so longest-first is LPT.  The estimate, in cycles of one workgroup:
  // phase A's tile-steps over 4 SIMDs at ~1 300 cycles each, phase B's messages at ~6
  hvec<int32_t> gorder(G);
  {
    std::vector<double> cost(G, 0.0);
    for (int g = 0; g < G; ++g) {
      double ts = 0;
      for (int64_t k = pstart[g]; k < pstart[g + 1]; k += 16) ts += ma.h_len[plist[k]];
      cost[g] = ts * 325.0 + (double)nmsg[g] * 6.0;
    }
    std::iota(gorder.begin(), gorder.end(), 0);
    std::stable_sort(gorder.begin(), gorder.end(), [&](int32_t x, int32_t y) { return cost[x] > cost[y]; });
  }
  // every state in LDS where the largest graph's fit, else the path states in global memory, else
  // also the sum MPs' CSR
  int form = IGN_RES_ALL_LDS;
  if (lds[0] > kResidentMaxDynLds || p->resident_path_global) {
    if (!p->resident_pg) return IGN_OK;
    form = lds[1] <= kResidentMaxDynLds ? IGN_RES_PATH_GLOBAL : IGN_RES_PATH_CSR_GLOBAL;
    if (lds[form] > kResidentMaxDynLds) return IGN_OK;
  }
  // the training forward's form: path states in global memory always (their versions)
  b->res_train_form = lds[1] <= kResidentMaxDynLds ? IGN_RES_PATH_GLOBAL : IGN_RES_PATH_CSR_GLOBAL;
  b->res_train_lds = lds[b->res_train_form];
  HIP_TRY(resident_prepare_device());
  std::vector<int64_t> pov(po.begin(), po.end());
  int rc;
  for (int s = 0; s < S; ++s) {
    std::vector<int64_t> sov(so[s]->begin(), so[s]->end());
    if ((rc = dev_upload(b, &b->d_res_src_off[s], sov))) return rc;
  }
  if ((rc = dev_upload(b, &b->d_res_path_off, pov)) || (rc = dev_upload(b, &b->d_res_urow_off, uo)) ||
      (rc = dev_upload(b, &b->d_res_ptile_off, ptile_off)) || (rc = dev_upload(b, &b->d_res_hdr, hdr)) ||
      (rc = dev_upload(b, &b->d_res_lmsg_off, lmsg_off)) || (rc = dev_upload(b, &b->d_res_lmsg_ptr, lmsg_ptr)) ||
      (rc = dev_upload(b, &b->d_res_lmsg_src, lmsg_src)) || (rc = dev_upload(b, &b->d_res_lorder, lorder)) ||
      (rc = dev_upload(b, &b->d_res_lnseg, lnseg)) || (rc = dev_upload(b, &b->d_res_lcode_off, lcode_off)) ||
      (rc = dev_upload(b, &b->d_res_hsb, hsb)) || (rc = dev_upload(b, &b->d_res_gorder, gorder)) ||
      (rc = dev_upload(b, &b->d_res_lcode, lcode)))
    return rc;
  b->res_lds = lds[form];
  b->res_form = form;
  b->res_graphs = G;
  // the cost model of one launch (ign_batch_resident_info)
  ign_resident_info_t& ri = b->res_info;
  ri = ign_resident_info_t{};
  ri.active = 1;
  ri.form = form;
  ri.lds_bytes = (int64_t)lds[form];
  ri.tile_steps = (int64_t)(tile_steps * p->T);
  ri.seg_rows = seg_rows;
  ri.messages = lmsg_off[G];
  double utiles = 0;
  for (int g = 0; g < G; ++g) utiles += (double)((Ls(0, g) + 15) / 16 + (Ls(1, g) + 15) / 16);
  ri.union_tiles = (int64_t)utiles;
  // compulsory: the features, tile headers, step codes and the sum CSR read once, the final states
  // written once
  const int64_t P = b->rows[path], Urows = uo[G];
  double feat = 4.0 * P * p->ents[path].feature_total;
  for (int s = 0; s < S; ++s) feat += 4.0 * b->rows[sh.src_ent[s]] * p->ents[sh.src_ent[s]].feature_total;
  ri.bytes_compulsory = feat + 4.0 * hdr.size() + 2.0 * (double)lcode.size() + 4.0 * lmsg_ptr.size() +
                        2.0 * lmsg_src.size() + 4.0 * 32 * (P + Urows);
  // global-path forms: every iteration moves each path row once in and out of the ordered update and
  // once per message into the sums (rows of 128 B) and reads the step codes again; the CSR-global
  // form also reads the message rows every iteration
  if (form != IGN_RES_ALL_LDS)
    ri.bytes_roundtrip = p->T * (128.0 * (2.0 * P + (double)lmsg_src.size()) + 2.0 * (double)lcode.size());
  if (form == IGN_RES_PATH_CSR_GLOBAL) ri.bytes_roundtrip += p->T * 2.0 * (double)lmsg_src.size();
  // B_stage of every MP (MPB::bytes), T times
  double stage = ma.bytes, mflops = ma.flops;
  for (int s = 0; s < S; ++s) {
    stage += b->mp[sh.sum_mp[s]].bytes;
    mflops += b->mp[sh.sum_mp[s]].flops;
  }
  ri.bytes_stage = p->T * stage;
  // the MPs' FLOPs per iteration plus the ordered MP's input projection of every union row
  ri.flops = p->T * (mflops + 2.0 * Urows * 32 * 96);
  // the matrix pipe: phase A's split-fp16 h.U (3 products x 3 gates x 2 tiles per tile-step), the
  // split-bf16 GRU step (2 x 36 per tile), the projection (3 gates x 2 x 6, T - 1 times), all
  // 16x16x32; iteration 0's projection on f32 MFMA (3 gates x 2 tiles x 8 k-steps per union tile;
  // the projection's tiles straddle the entities, ceil(U / 16) per graph)
  double ptiles = 0;
  for (int g = 0; g < G; ++g) ptiles += (double)((uo[g + 1] - uo[g] + 15) / 16);
  ri.mfma_bf16 = (p->T * (tile_steps * 18.0 + utiles * 72.0) + (p->T - 1) * utiles * 36.0) * kMfmaBf16Flops;
  ri.mfma_f32 = ptiles * 48.0 * kMfmaF32Flops;
  ri.workgroups = G;
  ri.graphs_per_workgroup = K;
  b->resident = true;
  return IGN_OK;
}

// ---------------------------------------------------------------------------------------------
// ign_batch_create's message lists for one (graph, source) of a plain MP (no interleave, attention or
// axis-2 concat), T the desc's index type: false when an index is out of range (the caller's checked
// loop then reports the first one)
extern "C++" template <class T>
static bool plain_messages(const T* __restrict as, const T* __restrict ad, const T* __restrict aq, int64_t n,
                           int64_t nsrc, int64_t ndst, int64_t rd, int64_t rs, int64_t slot_off, uint32_t sb, bool net,
                           int64_t e0, hvec<int32_t>& mdst, hvec<int32_t>& mpos, hvec<uint32_t>& mcode,
                           int64_t* __restrict fl) {
  bool bad = false;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t si = as[k], di = ad[k];
    bad |= (uint64_t)si >= (uint64_t)nsrc || (uint64_t)di >= (uint64_t)ndst;
    const int64_t dc = bad ? 0 : di;   // (no store outside the graph's flen range before the report)
    mdst.push_back((int32_t)(rd + dc));
    mpos.push_back((int32_t)(slot_off + (int64_t)aq[k]));
    mcode.push_back(sb | (uint32_t)(net ? e0 + k : rs + si));
    fl[dc] += 1;
  }
  return !bad;
}

int ign_batch_create(ign_plan* p, const ign_batch_desc* d, ign_batch** out) {
  if (!p || !d || !out) return fail(IGN_ERR_INVALID, "null argument");
  *out = nullptr;
  const int G = d->num_graphs;
  const int E = (int)p->ents.size();
  if (G <= 0) return fail(IGN_ERR_INVALID, "num_graphs must be > 0");
  int rc = ensure_device(p);
  if (rc) return rc;
  UploadScope scope("ign_batch_create");
  std::unique_ptr<ign_batch, void (*)(ign_batch*)> b(new ign_batch(), ign_batch_destroy);
  b->plan = p;
  b->pool = p->pool;
  b->G = G;
  b->rows.assign(E, 0);
  b->row_off.assign(E, std::vector<int64_t>(G + 1, 0));
  for (int e = 0; e < E; ++e) {
    for (int g = 0; g < G; ++g) {
      int64_t n = d->num_nodes[(int64_t)g * E + e];
      if (n < 0) return fail(IGN_ERR_INVALID, "graph %d: negative num_ for entity %d", g, e);
      b->row_off[e][g + 1] = b->row_off[e][g] + n;
    }
    b->rows[e] = b->row_off[e][G];
  }
  b->halo.assign(E, 0);
  if (d->halo_rows) {
    // a partition holds only its own destinations: the attention softmax normalises over all of the
    // graph's destinations per position (AUX:327-336), and the sorted updates pad per graph
    // (GM:477-543).  Sum / convolution MPs, with or without message networks, are destination-local.
    for (auto& mp : p->mps)
      if (mp.aggr == IGN_AGGR_ATTENTION || mp.sorted)
        return fail(IGN_ERR_UNSUPPORTED, "edge-cut partitions support sum and convolution MPs only (attention "
                    "normalises over the whole graph, AUX:327-336; ordered updates pad per graph, GM:477-543)");
    for (int e = 0; e < E; ++e) {
      if (d->halo_rows[e] < 0) return fail(IGN_ERR_INVALID, "entity %d: negative halo_rows", e);
      b->halo[e] = d->halo_rows[e];
      if (b->halo[e] && G != 1) return fail(IGN_ERR_INVALID, "halo rows need num_graphs == 1 (one partition)");
    }
  }
  for (int e = 0; e < E; ++e)
    if (b->rows[e] + b->halo[e] >= (int64_t)IGN_ROW_MASK) return fail(IGN_ERR_UNSUPPORTED, "entity %d: too many rows", e);
  // edge offsets per adjacency
  std::vector<hvec<int64_t>> eoff(p->n_adj, hvec<int64_t>(G + 1, 0));
  for (int a = 0; a < p->n_adj; ++a)
    for (int g = 0; g < G; ++g) {
      int64_t n = d->adj_edges[(int64_t)g * p->n_adj + a];
      if (n < 0) return fail(IGN_ERR_INVALID, "negative edge count");
      eoff[a][g + 1] = eoff[a][g] + n;
    }
  std::vector<IdxArr> asrc(p->n_adj), adst(p->n_adj), aseq(p->n_adj), ilx(p->n_il);   // ABI 13: int32 or int64
  if (d->index_bytes != 0 && d->index_bytes != 4 && d->index_bytes != 8)
    return fail(IGN_ERR_INVALID, "index_bytes %d (0 / 8: int64 index arrays, 4: int32)", (int)d->index_bytes);
  for (int a = 0; a < p->n_adj; ++a) {
    asrc[a] = IdxArr(d->adj_src[a], d->index_bytes);
    adst[a] = IdxArr(d->adj_dst[a], d->index_bytes);
    aseq[a] = IdxArr(d->adj_seq[a], d->index_bytes);
  }
  for (int i = 0; i < p->n_il; ++i) ilx[i] = IdxArr(d->interleave_idx[i], d->index_bytes);
  std::vector<hvec<int64_t>> ioff(p->n_il, hvec<int64_t>(G + 1, 0));
  for (int i = 0; i < p->n_il; ++i)
    for (int g = 0; g < G; ++g) ioff[i][g + 1] = ioff[i][g] + d->interleave_len[(int64_t)g * p->n_il + i];

  // features + state buffers
  b->d_feat.assign(E, nullptr);
  b->d_state[0].assign(E, nullptr);
  b->d_state[1].assign(E, nullptr);
  b->cur.assign(E, 0);
  for (int e = 0; e < E; ++e) {
    const int H = p->ents[e].hidden_dim, F = p->ents[e].feature_total;
    if (F > 0) {
      if (!d->features || !d->features[e]) return fail(IGN_ERR_INVALID, "entity %d: features missing", e);
      hvec<float> f(d->features[e], d->features[e] + b->rows[e] * F);
      if ((rc = dev_upload(b.get(), &b->d_feat[e], f))) return rc;
    }
    const int64_t sr = (b->rows[e] + b->halo[e]) * H;
    for (int k = 0; k < 2; ++k) {
      if ((rc = dev_alloc(b.get(), &b->d_state[k][e], sr))) return rc;
      if (b->halo[e]) HIP_TRY(hipMemsetAsync(b->d_state[k][e], 0, sr * sizeof(float), upload_stream()));   // halo defined before use
    }
  }

  // per-MP CSR / step tables
  static const bool build_prof = env_flag("IGN_BUILD_PROF", false);
  std::vector<double> t_mp;   // IGN_BUILD_PROF: the time up to the end of each MP's tables
  const double t_mp0 = build_prof ? now_ms() : 0.0;
  BuildMarks bm(env_flag("IGN_BUILD_PROF_FINE", false));   // IGN_BUILD_PROF_FINE=1: finer sections of each MP
  for (size_t mi = 0; mi < p->mps.size(); ++mi) {
    if (build_prof && mi > 0) t_mp.push_back(now_ms());
    const MPP& mp = p->mps[mi];
    const int S = (int)mp.src.size();
    const int dst = mp.dst;
    const int64_t ND = b->rows[dst];
    MPB mb;
    mb.sorted = mp.sorted;
    mb.n_dst = ND;
    // messages: (dst row, position, code), in source order then edge order
    hvec<int32_t> mdst;   // rows < IGN_ROW_MASK
    hvec<int32_t> mpos;   // < total_slots (checked)
    hvec<uint32_t> mcode;
    int64_t tot = 0;
    for (int s = 0; s < S; ++s) tot += eoff[mp.src[s].adjacency][G];
    mdst.reserve(tot);
    mpos.reserve(tot);
    mcode.reserve(tot);
    hvec<int64_t> flen(ND, 0);
    for (int g = 0; g < G; ++g) {
      int64_t slot_off = 0;  // sum of Lmax of previous sources in this graph (GM:533)
      hvec<int64_t> ilflat;
      if (mp.aggr == IGN_AGGR_INTERLEAVE) {
        // tf.stack([indices_a, indices_b]) then reshape [-1,1] (GM:518, AUX:433)
        int64_t len0 = -1;
        for (int s = 0; s < S; ++s) {
          int il = mp.src[s].interleave;
          int64_t n = ioff[il][g + 1] - ioff[il][g];
          if (len0 >= 0 && n != len0)
            return fail(IGN_ERR_INVALID, "graph %d: interleave index lists have different lengths (%lld vs %lld;"
                        " tf.stack fails, GM:518)", g, (long long)len0, (long long)n);
          len0 = n;
          for (int64_t k = ioff[il][g]; k < ioff[il][g + 1]; ++k) ilflat.push_back(ilx[il][k]);
        }
      }
      int64_t total_slots = 0;
      hvec<int64_t> lmax(S, 0);
      for (int s = 0; s < S; ++s) {
        const int a = mp.src[s].adjacency;
        const int64_t e0 = eoff[a][g], e1 = eoff[a][g + 1];
        if (e1 == e0)
          return fail(IGN_ERR_INVALID, "graph %d: adjacency slot %d has no edges (the reference's scatter_nd shape"
                      " max(seq)+1 is undefined, GM:484-490)", g, a);
        int64_t mx = -1;
        for (int64_t k = e0; k < e1; ++k) {
          int64_t sq = aseq[a][k];
          if (sq < 0) return fail(IGN_ERR_INVALID, "graph %d: negative seq value", g);
          mx = std::max(mx, sq);
        }
        lmax[s] = mx + 1;
        total_slots += lmax[s];
      }
      if (total_slots >= INT32_MAX) return fail(IGN_ERR_UNSUPPORTED, "graph %d: sequences too long", g);
      if (mp.feature_concat) {   // tf.concat on axis 2 needs every source's [N, Lmax] to match
        for (int s = 1; s < S; ++s)
          if (lmax[s] != lmax[0])
            return fail(IGN_ERR_INVALID, "graph %d: concat on axis 2 of sequences of length %lld and %lld "
                        "(ConcatOp dimension mismatch, GM:503)", g, (long long)lmax[0], (long long)lmax[s]);
        total_slots = lmax[0];
      }
      if (mp.aggr == IGN_AGGR_INTERLEAVE && (int64_t)ilflat.size() != total_slots)
        return fail(IGN_ERR_INVALID, "graph %d: interleave indices cover %lld slots but the messages need %lld"
                    " (scatter_nd shape mismatch, AUX:435)", g, (long long)ilflat.size(), (long long)total_slots);
      for (int s = 0; s < S; ++s) {
        const int a = mp.src[s].adjacency;
        const int se = mp.src[s].entity;
        const int64_t e0 = eoff[a][g], e1 = eoff[a][g + 1];
        const int64_t nsrc = b->row_off[se][g + 1] - b->row_off[se][g] + b->halo[se];   // halo: G == 1
        const int64_t ndst = b->row_off[dst][g + 1] - b->row_off[dst][g];
        // attention: comb_seq of source s > 0 is seq + that source's own in-degree (GM:539-540)
        hvec<int64_t> lens_s;
        if (mp.aggr == IGN_AGGR_ATTENTION && s > 0) {
          lens_s.assign(ndst, 0);
          for (int64_t k = e0; k < e1; ++k) {
            const int64_t di = adst[a][k];
            if (di >= 0 && di < ndst) lens_s[di]++;
          }
        }
        if (mp.aggr != IGN_AGGR_INTERLEAVE && mp.aggr != IGN_AGGR_ATTENTION && !mp.feature_concat) {
          // the common case (sum, ordered, convolution; no axis-2 concat): the loop below without its
          // per-message branches on the MP's kind, whose fields it reloaded on every message (the
          // stores may alias them), reading the desc's own index width.  An index out of range
          // reruns the checked loop, which reports the first one.
          const int64_t rd = b->row_off[dst][g], rs = b->row_off[se][g];
          const uint32_t sb = (uint32_t)s << IGN_SLOT_SHIFT;
          const bool net = !mp.nn[s].layers.empty();
          const bool ok = d->index_bytes == 4
              ? plain_messages(static_cast<const int32_t*>(asrc[a].p) + e0, static_cast<const int32_t*>(adst[a].p) + e0,
                               static_cast<const int32_t*>(aseq[a].p) + e0, e1 - e0, nsrc, ndst, rd, rs, slot_off, sb,
                               net, e0, mdst, mpos, mcode, flen.data() + rd)
              : plain_messages(d->adj_src[a] + e0, d->adj_dst[a] + e0, d->adj_seq[a] + e0, e1 - e0, nsrc, ndst, rd, rs,
                               slot_off, sb, net, e0, mdst, mpos, mcode, flen.data() + rd);
          if (ok) {
            slot_off += lmax[s];
            continue;
          }
        }
        for (int64_t k = e0; k < e1; ++k) {
          int64_t si = asrc[a][k], di = adst[a][k], sq = aseq[a][k];
          if (si < 0 || si >= nsrc) return fail(IGN_ERR_INVALID, "graph %d: src index %lld out of range [0,%lld)", g, (long long)si, (long long)nsrc);
          if (di < 0 || di >= ndst) return fail(IGN_ERR_INVALID, "graph %d: dst index %lld out of range [0,%lld)", g, (long long)di, (long long)ndst);
          int64_t pos = slot_off + sq;
          if (mp.aggr == IGN_AGGR_INTERLEAVE) {
            pos = ilflat[pos];
            if (pos < 0 || pos >= total_slots)
              return fail(IGN_ERR_INVALID, "graph %d: interleave index %lld outside [0,%lld) (scatter_nd, AUX:435)",
                          g, (long long)pos, (long long)total_slots);
          }
          if (mp.aggr == IGN_AGGR_ATTENTION) pos = sq + (s > 0 ? lens_s[di] : 0);
          if (mp.feature_concat) pos = sq;   // all sources share the positions (axis-2 concat)
          int64_t drow = b->row_off[dst][g] + di;
          mdst.push_back(drow);
          mpos.push_back(pos);
          // a message network's messages live per edge: the code addresses the edge (GM:440-475)
          const int64_t mrow = mp.nn[s].layers.empty() ? b->row_off[se][g] + si : k;
          mcode.push_back(((uint32_t)s << IGN_SLOT_SHIFT) | (uint32_t)mrow);
          // final_len = sum of lens over sources (GM:505/519/543); axis-2 concat keeps the first
          // source's lens (GM:503-505)
          if (!mp.feature_concat || s == 0) flen[drow] += 1;
        }
        slot_off += lmax[s];
      }
      if (mp.sorted) {
        // gather_nd(outputs, [d, final_len-1]) needs final_len <= sum of Lmax (AUX:793-795)
        int64_t max_flen = 0;
        for (int64_t r = b->row_off[dst][g]; r < b->row_off[dst][g + 1]; ++r) {
          if (flen[r] > total_slots)
            return fail(IGN_ERR_INVALID, "graph %d: destination row %lld has final_len %lld > %lld padded slots"
                        " (gather_nd out of range, AUX:793-795)", g, (long long)(r - b->row_off[dst][g]),
                        (long long)flen[r], (long long)total_slots);
          max_flen = std::max(max_flen, flen[r]);
        }
        // RNN(mask=tf.sequence_mask(final_len)) (AUX:785-790): the mask is max(final_len) wide, and
        // K.rnn unstacks it into a TensorList that its while loop reads at every one of the
        // total_slots time steps -> InvalidArgument at step max(final_len) when that is narrower
        // ("masked-RNN time length")
        if (b->row_off[dst][g + 1] > b->row_off[dst][g] && max_flen < total_slots)
          return fail(IGN_ERR_INVALID, "graph %d: sequence_mask(final_len) is %lld steps wide but the padded "
                      "sequence has %lld (K.rnn reads the mask TensorList past its end, AUX:785-790)", g,
                      (long long)max_flen, (long long)total_slots);
      }
    }
    for (int s = 0; s < S; ++s) {   // message networks: per-edge rows and parameters (GM:440-475)
      const MsgNN& nn = mp.nn[s];
      if (nn.layers.empty()) continue;
      const int a = mp.src[s].adjacency, se = mp.src[s].entity;
      const int64_t ne = eoff[a][G];
      if (ne >= (int64_t)IGN_ROW_MASK) return fail(IGN_ERR_UNSUPPORTED, "too many edges for a message network");
      hvec<int32_t> es(ne), ed(ne);
      for (int g = 0; g < G; ++g)
        for (int64_t k = eoff[a][g]; k < eoff[a][g + 1]; ++k) {
          es[k] = (int32_t)(b->row_off[se][g] + asrc[a][k]);
          ed[k] = (int32_t)(b->row_off[dst][g] + adst[a][k]);
        }
      mb.n_edges[s] = ne;
      if ((rc = dev_upload(b.get(), &mb.d_edge_src[s], es)) || (rc = dev_upload(b.get(), &mb.d_edge_dst[s], ed))) return rc;
      if (std::find(nn.inputs.begin(), nn.inputs.end(), (int)IGN_MSG_EDGE_PARAMS) != nn.inputs.end()) {
        if (!d->adj_params || !d->adj_params[a])
          return fail(IGN_ERR_INVALID, "message network of mp %zu reads edge_params but params_<adj> is missing", mi);
        hvec<float> prm(d->adj_params[a], d->adj_params[a] + ne * nn.param_dim);
        if ((rc = dev_upload(b.get(), &mb.d_edge_params[s], prm))) return rc;
      }
      if ((rc = dev_alloc(b.get(), &mb.d_msg_in[s], ne * nn.din_pad))) return rc;
      HIP_TRY(hipMemsetAsync(mb.d_msg_in[s], 0, ne * nn.din_pad * sizeof(float), upload_stream()));   // zero padding columns
      for (auto& dp : nn.layers) {
        float* f = nullptr;
        if ((rc = dev_alloc(b.get(), &f, ne * dp.out))) return rc;
        mb.d_msg_layer[s].push_back(f);
      }
    }
    bm.mark("messages");
    mb.edges = tot;
    b->edges_per_forward += tot * p->T;
    const CellP& cp = p->cells[mp.cell];
    const int H = cp.H, DIN = mp.din;

    hvec<int32_t> order(ND);
    std::iota(order.begin(), order.end(), 0);
    if (mp.sorted) {
      for (int64_t r = 0; r < ND; ++r)
        if (flen[r] == 0)   // AUX:793-795: gather_nd(outputs, [d, final_len-1]) with -1
          return fail(IGN_ERR_INVALID, "destination row %lld receives no message: the reference's sorted update"
                      " gathers position -1 (AUX:793-795)", (long long)r);
      sort_order(order, flen);
      bm.mark("sort");
      // combined projected table: source s occupies rows [src_off[s], src_off[s] + rows_s)
      int64_t trow = 0;
      for (int s = 0; s < S; ++s) {
        mb.src_off.push_back(trow);
        const int se = mp.src[s].entity;
        const int64_t rows_s = mp.nn[s].layers.empty() ? b->rows[se] + b->halo[se] : eoff[mp.src[s].adjacency][G];
        mb.src_rows.push_back(rows_s);
        trow += rows_s;
      }
      mb.zero_row = trow;
      auto table_row = [&](uint32_t code) -> int64_t {
        return mb.src_off[code >> IGN_SLOT_SHIFT] + (code & IGN_ROW_MASK);
      };
      // Step t of the destination at sorted position i is slot step_ptr[i] + t.  A slot holds its
      // message's table row, the zero row (a hole), or a pre-summed "multi" row when several
      // messages share the position (scatter_nd adds them); messages at positions >= final_len
      // are dropped (the masked RNN never reads them).  Multi rows are numbered in slot order and
      // list their messages in message order.  maxL + 8 trailing zero-row slots: the kernels read
      // codes past a row's end unconditionally.
      hvec<int32_t> len(ND), step_ptr(ND), multi_ptr(1, 0);
      hvec<int32_t> where(ND);
      int64_t steps = 0, maxL = 0;
      for (int64_t i = 0; i < ND; ++i) {
        const int64_t r = order[i];
        where[r] = (int32_t)i;
        len[i] = (int32_t)flen[r];
        step_ptr[i] = (int32_t)steps;
        maxL = std::max(maxL, flen[r]);
        steps += flen[r];
      }
      if (steps >= INT32_MAX) return fail(IGN_ERR_UNSUPPORTED, "MP too large");
      hvec<uint32_t> scode((size_t)(steps + maxL + 8), (uint32_t)mb.zero_row);
      hvec<int32_t> slot_of(mdst.size(), -1), scount(steps, 0);
      int64_t n_msgs = 0;
      for (size_t k = 0; k < mdst.size(); ++k) {
        const int64_t r = mdst[k];
        if (mpos[k] >= flen[r]) continue;
        const int64_t slot = step_ptr[where[r]] + mpos[k];
        slot_of[k] = (int32_t)slot;
        if (++scount[slot] == 1) scode[slot] = (uint32_t)table_row(mcode[k]);
        ++n_msgs;
      }
      hvec<uint32_t> multi_rows;
      hvec<int32_t> multi_of(steps, -1);
      for (int64_t slot = 0; slot < steps; ++slot)
        if (scount[slot] > 1) {
          multi_of[slot] = (int32_t)mb.n_multi;
          scode[slot] = (uint32_t)(mb.zero_row + 1 + mb.n_multi);
          multi_ptr.push_back(multi_ptr.back() + scount[slot]);
          mb.n_multi++;
        }
      if (mb.n_multi) {
        multi_rows.resize(multi_ptr.back());
        hvec<int32_t> fill(multi_ptr.begin(), multi_ptr.end() - 1);
        for (size_t k = 0; k < mdst.size(); ++k)
          if (slot_of[k] >= 0 && multi_of[slot_of[k]] >= 0)
            multi_rows[fill[multi_of[slot_of[k]]]++] = (uint32_t)table_row(mcode[k]);
      }
      bm.mark("slots");
      for (int64_t i = 0; i < ND; i += 16) mb.wave_steps += len[i];   // sorted: a tile's first row is its longest
      {   // the ordered update's tile headers: one 16-B load per position, no dependent code load
        const int64_t NDp = (ND + 15) / 16 * 16;
        hvec<int32_t> hdr((size_t)(4 * NDp));
        for (int64_t i = 0; i < NDp; ++i) {
          const bool v = i < ND;
          hdr[4 * i] = v ? order[i] : 0;
          hdr[4 * i + 1] = v ? len[i] : 0;
          hdr[4 * i + 2] = v ? step_ptr[i] : (int32_t)steps;
          hdr[4 * i + 3] = (int32_t)scode[v ? step_ptr[i] : steps];
        }
        if ((rc = dev_upload(b.get(), &mb.d_seq_hdr, hdr))) return rc;
      }
      bm.mark("headers");
      if (mb.zero_row + 1 + mb.n_multi >= (int64_t)UINT32_MAX) return fail(IGN_ERR_UNSUPPORTED, "MP too large");
      mb.n_steps = steps;
      mb.n_msgs = n_msgs;
      if ((rc = dev_upload(b.get(), &mb.d_order, order))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_len, len))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_step_ptr, step_ptr))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_step_code, scode))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_multi_ptr, multi_ptr))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_multi_rows, multi_rows))) return rc;
      mb.h_order = std::move(order);
      mb.h_len = std::move(len);
      mb.h_step_ptr = std::move(step_ptr);
      mb.h_step_code = std::move(scode);
      mb.h_multi_ptr = std::move(multi_ptr);
      mb.h_multi_rows = std::move(multi_rows);
      const int64_t tfloats = (mb.zero_row + 1 + mb.n_multi) * 3LL * H;
      if ((rc = dev_alloc(b.get(), &mb.d_table, tfloats))) return rc;
      HIP_TRY(hipMemsetAsync(mb.d_table, 0, (tfloats + 256) * sizeof(float), upload_stream()));   // zero row stays zero
      // per launch of the recurrence: h.U + gates per step; one projected row (3H floats) per step
      // FLOPs executed (fp32-equivalent): h.U + gates per step (x.W is hoisted into project);
      // bytes per SURVEY §8d, B_stage = E (4 + 4H) + 2 N_d 4H + 4 (N_d + 1): one message row and
      // code per step, the state read and written once per destination
      mb.flops = (double)steps * (2.0 * H * 3 * H + 14.0 * H);
      mb.bytes = (double)steps * (4.0 * H + 4) + (double)ND * 8.0 * H + 4.0 * (ND + 1);
      b->gru_steps += steps * p->T;
      bm.mark("uploads");
    } else {
      sort_order(order, flen);
      // edge-cut partitions: destinations reading a halo row go last (they wait for the exchange)
      // (a message network's codes address edges, and its per-edge pass reads every source row
      // before any destination runs: no interior destinations then)
      bool nets = false;
      for (auto& nn : mp.nn) nets = nets || !nn.layers.empty();
      bool halo = false;
      for (auto& sd : mp.src) halo = halo || b->halo[sd.entity] > 0;
      hvec<char> bnd(ND, nets && halo ? 1 : 0);
      for (size_t k = 0; k < mdst.size() && !nets; ++k) {
        const uint32_t c = mcode[k];
        const int se = mp.src[c >> IGN_SLOT_SHIFT].entity;
        if ((int64_t)(c & IGN_ROW_MASK) >= b->rows[se]) bnd[mdst[k]] = 1;
      }
      std::stable_partition(order.begin(), order.end(), [&](int32_t r) { return !bnd[r]; });
      bm.mark("sort");
      mb.n_interior = std::count(bnd.begin(), bnd.end(), 0);
      hvec<int32_t> where(ND);
      for (int64_t i = 0; i < ND; ++i) where[order[i]] = (int32_t)i;
      hvec<int32_t> ptr(ND + 1, 0);
      for (size_t k = 0; k < mdst.size(); ++k) ptr[where[mdst[k]] + 1]++;
      for (int64_t i = 0; i < ND; ++i) ptr[i + 1] += ptr[i];
      hvec<uint32_t> msrc(mdst.size());
      hvec<int32_t> csr_pos(mp.aggr == IGN_AGGR_ATTENTION ? mdst.size() : 0);   // message -> CSR slot
      {
        hvec<int32_t> fill(ptr.begin(), ptr.end() - 1);
        for (size_t k = 0; k < mdst.size(); ++k) {
          const int32_t q = fill[where[mdst[k]]]++;
          if (!csr_pos.empty()) csr_pos[k] = q;
          msrc[q] = mcode[k];
        }
      }
      if (mp.aggr == IGN_AGGR_ATTENTION) {
        // dense (destination, position) cells of the scatter_nd (AUX:327-331); duplicates share one
        // cell.  Groups = (graph, position): the softmax runs over a graph's destinations (AUX:336)
        hvec<int> gof(ND);
        for (int g = 0; g < G; ++g)
          for (int64_t r = b->row_off[dst][g]; r < b->row_off[dst][g + 1]; ++r) gof[r] = g;
        hvec<int64_t> key(mdst.size());
        hvec<int64_t> gmax(G, 0);
        for (size_t k = 0; k < mdst.size(); ++k) gmax[gof[mdst[k]]] = std::max<int64_t>(gmax[gof[mdst[k]]], mpos[k] + 1);
        hvec<int64_t> gbase(G + 1, 0);   // group index base per graph
        for (int g = 0; g < G; ++g) gbase[g + 1] = gbase[g] + gmax[g];
        hvec<size_t> ord(mdst.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) {
          const int64_t gx = gbase[gof[mdst[x]]] + mpos[x], gy = gbase[gof[mdst[y]]] + mpos[y];
          return gx != gy ? gx < gy : mdst[x] < mdst[y];
        });
        hvec<int32_t> group_ptr(gbase[G] + 1, 0), group_empty(gbase[G], 0), cell_dst, cell_ptr(1, 0), cell_msgs;
        for (size_t q = 0; q < ord.size();) {
          const size_t k = ord[q];
          const int64_t grp = gbase[gof[mdst[k]]] + mpos[k];
          size_t q2 = q;
          while (q2 < ord.size() && mdst[ord[q2]] == mdst[k] && mpos[ord[q2]] == mpos[k]) cell_msgs.push_back(csr_pos[ord[q2++]]);
          cell_dst.push_back((int32_t)mdst[k]);
          cell_ptr.push_back((int32_t)cell_msgs.size());
          group_ptr[grp + 1]++;
          q = q2;
        }
        for (int64_t q = 0; q < gbase[G]; ++q) group_ptr[q + 1] += group_ptr[q];
        for (int g = 0; g < G; ++g)
          for (int64_t pq = 0; pq < gmax[g]; ++pq) {
            const int64_t grp = gbase[g] + pq;
            group_empty[grp] = (int32_t)((b->row_off[dst][g + 1] - b->row_off[dst][g]) - (group_ptr[grp + 1] - group_ptr[grp]));
          }
        mb.n_groups = gbase[G];
        mb.n_cells = (int64_t)cell_dst.size();
        if ((rc = dev_upload(b.get(), &mb.d_group_ptr, group_ptr)) || (rc = dev_upload(b.get(), &mb.d_group_empty, group_empty)) ||
            (rc = dev_upload(b.get(), &mb.d_cell_dst, cell_dst)) || (rc = dev_upload(b.get(), &mb.d_cell_ptr, cell_ptr)) ||
            (rc = dev_upload(b.get(), &mb.d_cell_msgs, cell_msgs)))
          return rc;
        if ((rc = dev_alloc(b.get(), &mb.d_msg_w, (int64_t)mdst.size())) || (rc = dev_alloc(b.get(), &mb.d_ecell, mb.n_cells)) ||
            (rc = dev_alloc(b.get(), &mb.d_s_dst, ND)))
          return rc;
        for (int s = 0; s < S; ++s) {
          const int se = mp.src[s].entity;
          const int64_t rows_s = mp.nn[s].layers.empty() ? b->rows[se] + b->halo[se] : eoff[mp.src[s].adjacency][G];
          if ((rc = dev_alloc(b.get(), &mb.d_s_src[s], rows_s))) return rc;
        }
      }
      // windowed sum: one workgroup per (graph, chunk of <= 256 destinations by message count), the
      // destination's source rows ascending (a fixed summation order), LDS windows over the graph's
      // source rows; the GRU step then reads x through an identity CSR over the same order
      // (small graphs only: a workgroup walks all of its graph's windows, at most 4 of them)
      int64_t max_src_rows = 0;
      if (S == 1)
        for (int g = 0; g < G; ++g)
          max_src_rows = std::max(max_src_rows, b->row_off[mp.src[0].entity][g + 1] - b->row_off[mp.src[0].entity][g]);
      const int64_t win_rows = DIN == 16 ? 2400 : DIN == 32 ? 1200 : 600;   // sum_win_kernel's windows
      // IGN_SUM_WINDOW: -1 auto, 0 off below 128 messages (one lane group per destination walks its
      // messages in the GRU-step kernel), 1 windowed, 2 segmented for every destination.  Auto takes the segmented
      // sum (one wave per destination) for the destinations whose lane walk would be a long dependent
      // chain: >= 64 messages (seg_min_messages; Q-size's path -> node update, ~140 per node: 4.36-4.39
      // ms/step against 5.19 windowed and 5.51 lane-walk in round 4).  The rule reads each
      // destination's own in-degree, a property of its graph, so a graph's predictions stay bitwise
      // the same alone and in any batch (the two kernels add a destination's messages in different
      // orders), and the graph-resident forward takes the same order per row (resident.hip B1).
      bm.mark("csr");
      const bool window = p->sum_window == 1;
      int64_t n_seg = 0;   // order is sorted by message count, descending: the segmented rows lead
      if (p->sum_window == 0 && ND > 0 && ptr[1] - ptr[0] >= kSegMinMessages)   // (order: by count, descending)
        return fail(IGN_ERR_UNSUPPORTED, "IGN_SUM_WINDOW=0 (every sum a lane walk): mp %d has a destination of %lld "
                    "messages; a float32 chain of >= %lld terms leaves the fp32 class, so this switch is for batches "
                    "below that", (int)mi, (long long)(ptr[1] - ptr[0]), (long long)kSegMinMessages);
      if (!window && !halo)
        while (n_seg < ND && ptr[n_seg + 1] - ptr[n_seg] >= seg_min_messages(p)) ++n_seg;
      const bool seg = n_seg > 0;
      if (window && mp.aggr == IGN_AGGR_SUM && S == 1 && mp.nn[0].layers.empty() &&
          b->halo[mp.src[0].entity] == 0 && (DIN == 16 || DIN == 32 || DIN == 64) && max_src_rows <= 4 * win_rows) {
        const int se = mp.src[0].entity;
        hvec<int64_t> dstart(ND + 1, 0);
        for (size_t k = 0; k < mdst.size(); ++k) dstart[mdst[k] + 1]++;
        for (int64_t r = 0; r < ND; ++r) dstart[r + 1] += dstart[r];
        hvec<int32_t> rows_by(mdst.size());
        {
          hvec<int64_t> fill(dstart.begin(), dstart.end() - 1);
          for (size_t k = 0; k < mdst.size(); ++k) rows_by[fill[mdst[k]]++] = (int32_t)(mcode[k] & IGN_ROW_MASK);
        }
        for (int64_t r = 0; r < ND; ++r) std::sort(rows_by.begin() + dstart[r], rows_by.begin() + dstart[r + 1]);
        hvec<int64_t> wg;
        hvec<int32_t> wdst, wptr(1, 0), wsrc;
        wdst.reserve(ND);
        wsrc.reserve(mdst.size());
        for (int g = 0; g < G; ++g) {
          hvec<int32_t> ds;
          for (int64_t r = b->row_off[dst][g]; r < b->row_off[dst][g + 1]; ++r) ds.push_back((int32_t)r);
          std::stable_sort(ds.begin(), ds.end(), [&](int32_t x, int32_t y) { return flen[x] > flen[y]; });
          for (size_t c0 = 0; c0 < ds.size(); c0 += 256) {
            const size_t c1 = std::min(ds.size(), c0 + 256);
            wg.push_back((int64_t)wdst.size());
            wg.push_back((int64_t)(wdst.size() + (c1 - c0)));
            wg.push_back(b->row_off[se][g]);
            wg.push_back(b->row_off[se][g + 1]);
            for (size_t q = c0; q < c1; ++q) {
              const int32_t r = ds[q];
              wdst.push_back(r);
              wsrc.insert(wsrc.end(), rows_by.begin() + dstart[r], rows_by.begin() + dstart[r + 1]);
              wptr.push_back((int32_t)wsrc.size());
            }
          }
        }
        hvec<int32_t> id_ptr(ND + 1);
        hvec<uint32_t> id_src(ND);
        for (int64_t i = 0; i <= ND; ++i) id_ptr[i] = (int32_t)i;
        for (int64_t i = 0; i < ND; ++i) id_src[i] = (uint32_t)order[i];   // slot 0: the x table
        mb.n_win_wg = (int64_t)wg.size() / 4;
        if ((rc = dev_upload(b.get(), &mb.d_win_wg, wg)) || (rc = dev_upload(b.get(), &mb.d_win_dst, wdst)) ||
            (rc = dev_upload(b.get(), &mb.d_win_ptr, wptr)) || (rc = dev_upload(b.get(), &mb.d_win_src, wsrc)) ||
            (rc = dev_upload(b.get(), &mb.d_id_ptr, id_ptr)) || (rc = dev_upload(b.get(), &mb.d_id_src, id_src)) ||
            (rc = dev_alloc(b.get(), &mb.d_xsum, std::max<int64_t>(ND, 1) * DIN)))
          return rc;
      } else if (seg && mp.aggr == IGN_AGGR_SUM && S == 1 && mp.nn[0].layers.empty() && b->halo[mp.src[0].entity] == 0 &&
                 (DIN == 16 || DIN == 32 || DIN == 64)) {
        // segmented sum (sum_seg_kernel over the MP's own CSR, one wave per destination) for order
        // positions [0, n_seg), then the GRU step over a mixed CSR: those positions read their x
        // from the xsum table (one message, slot 1; the lane walk adds it to zero exactly), the
        // others their own messages (slot 0)
        hvec<int32_t> id_ptr(ND + 1, 0);
        hvec<uint32_t> id_src;
        id_src.reserve((size_t)(n_seg + (ptr[ND] - ptr[n_seg])));
        for (int64_t i = 0; i < ND; ++i) {
          if (i < n_seg) id_src.push_back((1u << IGN_SLOT_SHIFT) | (uint32_t)order[i]);
          else id_src.insert(id_src.end(), msrc.begin() + ptr[i], msrc.begin() + ptr[i + 1]);
          id_ptr[i + 1] = (int32_t)id_src.size();
        }
        mb.sum_seg = true;
        mb.n_seg = n_seg;
        if ((rc = dev_upload(b.get(), &mb.d_id_ptr, id_ptr)) || (rc = dev_upload(b.get(), &mb.d_id_src, id_src)) ||
            (rc = dev_alloc(b.get(), &mb.d_xsum, std::max<int64_t>(ND, 1) * DIN)))
          return rc;
      }
      mb.n_msgs = (int64_t)msrc.size();
      if ((rc = dev_upload(b.get(), &mb.d_order, order))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_msg_ptr, ptr))) return rc;
      if ((rc = dev_upload(b.get(), &mb.d_msg_src, msrc))) return rc;
      mb.h_order = std::move(order);
      mb.h_msg_ptr = std::move(ptr);
      mb.h_msg_src = std::move(msrc);
      mb.flops = (double)ND * gru_flops(DIN, H) + (double)mb.n_msgs * DIN;
      mb.bytes = (double)mb.n_msgs * (4.0 * DIN + 4) + (double)ND * (8.0 * H + 8);
      b->gru_steps += ND * p->T;
    }
    b->mp.push_back(std::move(mb));
  }

  // readout buffers (the resident forward's tables are built by the first ign_forward: a batch that
  // only trains or steps MP by MP never pays for them)
  bm.mark("mp-rest");
  if ((rc = readout_batch(p, b.get(), d))) return rc;
  bm.mark("readout");
  const int64_t P = space_rows(p, b.get(), p->ro_t[p->ro_in[0]]);
  b->n_pred = P;
  b->out_units = p->dense.back().out;
  if (p->ro_in.size() > 1 && (rc = dev_alloc(b.get(), &b->d_ro_in, P * p->ro_width))) return rc;
  if (!p->fused_readout) {
    for (size_t l = 0; l + 1 < p->dense.size(); ++l) {
      float* t = nullptr;
      if ((rc = dev_alloc(b.get(), &t, P * p->dense[l].out))) return rc;
      b->d_ro_tmp.push_back(t);
    }
  }
  if ((rc = dev_alloc(b.get(), &b->d_pred, P * b->out_units))) return rc;
  // the resident tables here, on the building thread, not at the first forward: a training loop's
  // builders run ahead of the step, and the step's thread would otherwise build them inside the step
  // (fresh 512 x synth50 batches: 28 -> 56 ms per step once the training forward went resident)
  const double t_res0 = build_prof ? now_ms() : 0.0;
  if (env_flag("IGN_RESIDENT_EAGER", true) && (rc = resident_tables(p, b.get()))) return rc;
  if (build_prof) {
    std::string s;
    double prev = t_mp0;
    for (size_t i = 0; i < t_mp.size(); ++i) {
      s += " mp" + std::to_string(i) + " " + std::to_string(t_mp[i] - prev).substr(0, 6);
      prev = t_mp[i];
    }
    fprintf(stderr, "[ign-build] batch sections:%s mp%zu+readout %.2f, resident tables %.2f ms\n", s.c_str(),
            t_mp.size(), t_res0 - prev, now_ms() - t_res0);
  }
  bm.mark("alloc+resident");
  bm.print("ign_batch_create fine");
  HIP_TRY(hipStreamSynchronize(upload_stream()));   // every clear has landed before the batch is used
  HIP_TRY(upload_flush());                           // (and every staged copy)
  *out = b.release();
  return IGN_OK;
}

void ign_batch_destroy(ign_batch* b) {
  if (!b) return;
  static const bool prof = env_flag("IGN_BUILD_PROF", false);
  const double t0 = prof ? now_ms() : 0.0;
  if (b->plan) {
    hipSetDevice(b->plan->device);
    // With the block cache every released block carries an event recorded on the plan stream
    // (pool_release), so the host need not wait here and the next step can be queued behind this
    // one.  Without it (IGN_POOL=0) pool_release waits itself; a captured graph is destroyed only
    // once its launches have finished.
    if (b->plan->stream && (b->graph || !pool_enabled(b->pool.get()))) hipStreamSynchronize(b->plan->stream);
  }
  if (b->graph) hipGraphExecDestroy(b->graph);
  const double t1 = prof ? now_ms() : 0.0;
  if (b->train) train_state_destroy(b->train);
  const double t2 = prof ? now_ms() : 0.0;
  if (b->pool) pool_release(b->pool.get(), b->allocs, b->plan ? b->plan->stream : nullptr);
  const double t3 = prof ? now_ms() : 0.0;
  delete b;
  if (prof)
    fprintf(stderr, "[ign-build] ign_batch_destroy: %.2f ms (sync %.2f, training state %.2f, blocks %.2f, host %.2f)\n",
            now_ms() - t0, t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
}

int ign_plan_trim_cache(ign_plan* p) {
  if (!p) return fail(IGN_ERR_INVALID, "null argument");
  if (p->pool) pool_trim_idle(p->pool.get());
  host_cache_trim();
  return IGN_OK;
}

int ign_batch_info(const ign_batch* b, ign_batch_info_t* o) {
  if (!b || !o) return fail(IGN_ERR_INVALID, "null argument");
  std::memset(o, 0, sizeof(*o));
  o->num_graphs = b->G;
  o->predictions = b->n_pred;
  o->output_units = b->out_units;
  o->edges_per_forward = b->edges_per_forward;
  o->gru_steps_per_forward = b->gru_steps;
  for (size_t e = 0; e < b->rows.size() && e < 8; ++e) o->rows[e] = b->rows[e];
  return IGN_OK;
}

int ign_batch_resident_info(const ign_batch* b, ign_resident_info_t* o) {
  if (!b || !o) return fail(IGN_ERR_INVALID, "null argument");
  *o = b->resident ? b->res_info : ign_resident_info_t{};
  return IGN_OK;
}

int ign_batch_predictions(ign_batch* b, const float** ptr) {
  if (!b || !ptr) return fail(IGN_ERR_INVALID, "null argument");
  *ptr = b->d_pred;
  return IGN_OK;
}

// ---------------------------------------------------------------------------------------------
namespace {

struct Timer {
  ign_plan* p;
  bool on = false;
  void begin(int kind, double flops, double bytes, double mfma_bf16 = 0, double mfma_f32 = 0) {
    on = p->timing && ((p->timing_kinds >> kind) & 1u);
    if (!on) return;
    if (p->ev_slot >= kMaxPendingEvents) flush_timing(p);
    const int slot = p->ev_slot;
    size_t need = 2 * (slot + 1);
    while (p->ev.size() < need) {
      hipEvent_t e;
      hipEventCreate(&e);
      p->ev.push_back(e);
    }
    if ((int)p->ev_kind.size() <= slot) {
      p->ev_kind.resize(slot + 1);
      p->ev_cost.resize(slot + 1);
    }
    p->ev_kind[slot] = kind;
    p->ev_cost[slot] = EvCost{flops, bytes, mfma_bf16, mfma_f32};
    hipEventRecord(p->ev[2 * slot], p->stream);
  }
  void end() {
    if (!on) return;
    hipEventRecord(p->ev[2 * p->ev_slot + 1], p->stream);
    ++p->ev_slot;
  }
};

// message network of one source: per-edge [inputs...] then the Dense stack into d_msg_layer[s]
int message_net_fwd(ign_plan* p, const MsgNN& nn, const MPB& mb, int s, const float* src_state,
                    const float* dst_state, hipStream_t st) {
  MsgGatherArgs g{};
  g.out = mb.d_msg_in[s];
  g.n = mb.n_edges[s];
  g.ld = nn.din_pad;
  g.nparts = (int)nn.inputs.size();
  int col = 0;
  for (int q = 0; q < g.nparts; ++q) {
    const int kind = nn.inputs[q];
    g.col[q] = col;
    g.width[q] = nn.widths[q];
    if (kind == IGN_MSG_HS_SOURCE) { g.base[q] = src_state; g.rows[q] = mb.d_edge_src[s]; }
    else if (kind == IGN_MSG_HS_DEST) { g.base[q] = dst_state; g.rows[q] = mb.d_edge_dst[s]; }
    else { g.base[q] = mb.d_edge_params[s]; g.rows[q] = nullptr; }
    col += g.width[q];
  }
  HIP_TRY(launch_msg_gather(g, st));
  const float* in = mb.d_msg_in[s];
  int stride = nn.din_pad;
  for (size_t l = 0; l < nn.layers.size(); ++l) {
    const DenseP& dp = nn.layers[l];
    const bool mfma = dp.pk_w >= 0;
    const int K = l == 0 ? (mfma ? nn.din_pad : nn.din) : dp.in;
    HIP_TRY(launch_dense_fwd(in, mb.n_edges[s], K, stride, mfma ? p->d_packed + dp.pk_w : nullptr,
                             p->d_params + dp.off_w, dp.use_bias ? p->d_params + dp.off_b : nullptr, dp.out, dp.act,
                             mb.d_msg_layer[s][l], st));
    in = mb.d_msg_layer[s][l];
    stride = dp.out;
  }
  return IGN_OK;
}

int check_pb(ign_plan* p, ign_batch* b) {
  if (!p || !b) return fail(IGN_ERR_INVALID, "null argument");
  if (b->plan != p) return fail(IGN_ERR_INVALID, "batch was created for another plan");
  if (!p->params_set) return fail(IGN_ERR_INVALID, "parameters not set (ign_plan_set_params)");
  return set_device(p->device);
}

}  // namespace

int ign_forward_begin(ign_plan* p, ign_batch* b) {
  int rc = check_pb(p, b);
  if (rc) return rc;
  Timer tm{p};
  for (int e = 0; e < (int)p->ents.size(); ++e) {   // GM:396-400 (owned rows; halo rows come from peers)
    const int H = p->ents[e].hidden_dim, F = p->ents[e].feature_total;
    tm.begin(K_INIT, 0, (double)b->rows[e] * (4.0 * F + 4.0 * H));
    HIP_TRY(launch_init_state(b->d_state[0][e], b->d_feat[e], b->rows[e], H, F, p->stream));
    tm.end();
    b->cur[e] = 0;
  }
  return IGN_OK;
}

// f32 MFMA FLOPs of a sum update's GRU step (sum_gru_kernel / sum_gru_lds: 3 gates x H/16 unit tiles x
// (DIN + H)/4 k-steps per 16-row tile)
static double sum_mfma_f32(int64_t n, int din, int H) {
  return (double)((n + 15) / 16) * 3 * (H / 16) * ((din + H) / 4) * kMfmaF32Flops;
}

// The ordered MP whose input projection sum MP mi can produce in its epilogue (sum_gru_g32), or -1,
// and in *slot the source of that MP whose table rows it fills: the next MP (cyclically, within this
// forward) that touches mi's destination entity reads it as exactly one of its sources, with the
// projection sum_gru_g32 forms (32 -> 3 x 32, no message network, no feature concat), and every row
// of the entity is one of mi's destinations (no halo rows).  A multi-source reader (Q-size's
// {link, node} -> path interleave) gets each source's rows from the sum update of that source.
static int fused_proj_target(const ign_plan* p, const ign_batch* b, int mi, int* slot) {
  const MPP& mp = p->mps[mi];
  const int e = mp.dst, n = (int)p->mps.size();
  if (mp.sorted || mp.aggr != IGN_AGGR_SUM || mp.feature_concat || mp.din != 32 || p->cells[mp.cell].H != 32 ||
      b->halo[e] > 0)
    return -1;
  for (const MsgNN& nn : mp.nn)
    if (!nn.layers.empty()) return -1;
  for (int k = 1; k <= n; ++k) {
    const int m2 = (mi + k) % n;
    if (m2 <= mi && b->fuse_last_iter) return -1;   // the next reader runs in no later iteration
    const MPP& q = p->mps[m2];
    int reads = 0, s_e = -1;
    for (size_t s = 0; s < q.src.size(); ++s)
      if (q.src[s].entity == e) {
        ++reads;
        s_e = (int)s;
      }
    if (!reads && q.dst != e) continue;
    const CellP& qc = p->cells[q.cell];
    if (m2 == mi || reads != 1 || !q.sorted || q.src.size() > 8 || q.feature_concat || !q.nn[s_e].layers.empty() ||
        q.din != 32 || qc.H != 32 || qc.pk_wbf < 0)
      return -1;
    *slot = s_e;
    return m2;
  }
  return -1;
}

int ign_forward_mp(ign_plan* p, ign_batch* b, int32_t mi, int32_t part) {
  int rc = check_pb(p, b);
  if (rc) return rc;
  if (mi < 0 || mi >= (int)p->mps.size()) return fail(IGN_ERR_INVALID, "mp index %d out of range", mi);
  if (part < IGN_PART_ALL || part > IGN_PART_BOUNDARY) return fail(IGN_ERR_INVALID, "part %d", part);
  hipStream_t st = p->stream;
  Timer tm{p};
  const MPP& mp = p->mps[mi];
  const MPB& mb = b->mp[mi];
  const CellP& cp = p->cells[mp.cell];
  SrcBases sbases{};
  for (size_t s = 0; s < mp.src.size(); ++s) {
    int se = mp.src[s].entity;
    sbases.base[s] = b->d_state[b->cur[se]][se];
  }
  const int dst = mp.dst;
  const float* hin = b->d_state[b->cur[dst]][dst];
  float* hout = b->d_state[1 - b->cur[dst]][dst];
  for (size_t s = 0; s < mp.src.size(); ++s) {   // message-creation networks (GM:440-475)
    const MsgNN& nn = mp.nn[s];
    if (nn.layers.empty()) continue;
    // the per-edge network reads halo rows: it must run after the exchange, not beside it
    if (part != IGN_PART_ALL) return fail(IGN_ERR_UNSUPPORTED, "interior/boundary split with a message network");
    if ((rc = message_net_fwd(p, nn, mb, (int)s, sbases.base[s], hin, st))) return rc;
  }
  for (size_t s = 0; s < mp.src.size(); ++s)
    if (!mp.nn[s].layers.empty()) sbases.base[s] = mb.d_msg_layer[s].back();
  if (mp.sorted) {
    if (part != IGN_PART_ALL) return fail(IGN_ERR_UNSUPPORTED, "interior/boundary split is for sum MPs only");
    const int W3 = 3 * cp.H;
    // sources whose table rows the previous sum updates' epilogues already formed (bit s)
    const int projected = b->fuse_ok ? b->proj_ready[mi] : 0;
    b->proj_ready[mi] = 0;
    for (size_t s = 0; s < mp.src.size(); ++s) {
      if (projected >> s & 1) continue;
      const int64_t rs = mb.src_rows[s];
      const int sdin_t = mp.feature_concat ? p->ents[mp.src[s].entity].hidden_dim : mp.din;
      tm.begin(K_PROJECT, 2.0 * rs * mp.din * W3, (double)rs * (4.0 * mp.din + 4.0 * W3), 0,
               (double)((rs + 15) / 16) * 3 * (cp.H / 16) * (sdin_t / 4) * kMfmaF32Flops);
      const int sdin = mp.feature_concat ? p->ents[mp.src[s].entity].hidden_dim : mp.din;
      const float* wp = mp.feature_concat ? p->d_packed + mp.pk_slice[s] : p->d_packed + cp.pk_w;
      HIP_TRY(launch_project(sbases.base[s], rs, wp, p->d_packed + cp.pk_b, mb.d_table + mb.src_off[s] * W3,
                             s == 0 ? mb.d_table + mb.zero_row * W3 : nullptr, sdin, cp.H, st));
      tm.end();
    }
    if (mb.n_multi) {
      tm.begin(K_OTHER, 0, 0);
      HIP_TRY(launch_multi_sum(mb.d_table, mb.zero_row + 1, mb.n_multi, mb.d_multi_ptr, mb.d_multi_rows, W3,
                               mb.d_table + mb.zero_row * W3, st));
      tm.end();
    }
    SeqGruArgs a{hin, hout, mb.d_table, mb.d_order, mb.d_len, mb.d_step_ptr, mb.d_step_code,
                 p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, mb.n_dst, p->xcd_remap};
    if (cp.pk_ubf >= 0) a.Ubf = p->d_packed + cp.pk_ubf;
    if (cp.pk_uh >= 0) a.Uh = p->d_packed + cp.pk_uh;
    a.hdr = mb.d_seq_hdr;
    {   // MFMAs per wave step: split-fp16 / split-bf16 (variants 6, 7 / 4, 5; H = 32 / 64) passes x
        // 3 gates x H/16 x H/32 on the 16x16x32 pipe; f32 (seq_gru2) 3 gates x H/16 x H/4
      const int v = p->seq_variant;
      const int passes = v == 6 ? 3 : 6;
      const bool bf = v >= 4 && (cp.H == 32 || cp.H == 64) && a.Ubf;
      const double ws = (double)mb.wave_steps;
      tm.begin(K_SEQ, mb.flops, mb.bytes,
               bf ? ws * passes * 3 * (cp.H / 16) * (cp.H / 32) * kMfmaBf16Flops : 0,
               bf ? 0 : ws * 3 * (cp.H / 16) * (cp.H / 4) * kMfmaF32Flops);
    }
    HIP_TRY(launch_seq_gru(a, cp.H, p->seq_variant, st));
    tm.end();
  } else {
    // destinations [first, first + count) of the order array
    const int64_t first = part == IGN_PART_BOUNDARY ? mb.n_interior : 0;
    const int64_t count = part == IGN_PART_INTERIOR ? mb.n_interior
                        : part == IGN_PART_BOUNDARY ? mb.n_dst - mb.n_interior : mb.n_dst;
    if (mp.aggr == IGN_AGGR_ATTENTION) {   // AUX:287-343: scores, then the axis-0 softmax weights
      // a softmax group spans interior and boundary destinations: no split
      if (part != IGN_PART_ALL) return fail(IGN_ERR_UNSUPPORTED, "interior/boundary split with attention");
      tm.begin(K_OTHER, 0, 0);
      if ((rc = attention_weights(p, b, mp, mb, sbases.base, hin, st))) return rc;
      tm.end();
    }
    if (count > 0) {
      // windowed or segmented aggregation (sum MPs over all destinations): the sum kernel writes x,
      // then the GRU step reads it through an identity CSR (one message per destination: x itself)
      const bool pre = (mb.n_win_wg > 0 || mb.sum_seg) && part == IGN_PART_ALL && mp.aggr == IGN_AGGR_SUM;
      SrcBases xb{};   // windowed: every x from the xsum table (slot 0); segmented: the mixed CSR's slot 1
      if (mb.sum_seg) {
        xb = sbases;
        xb.base[1] = mb.d_xsum;
      } else {
        xb.base[0] = mb.d_xsum;
      }
      SumGruArgs a{hin, hout, pre ? xb : sbases, pre ? mb.d_order : mb.d_order + first,
                   pre ? mb.d_id_ptr : mb.d_msg_ptr + first, pre ? mb.d_id_src : mb.d_msg_src,
                   p->d_packed + cp.pk_w, p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, count, p->xcd_remap};
      if (mp.aggr == IGN_AGGR_ATTENTION) a.msg_w = mb.d_msg_w;
      int sv = std::min(p->sum_variant, 7);
      if (mp.aggr == IGN_AGGR_SUM && cp.pk_wbf >= 0 && cp.pk_ubf >= 0 && mp.din == cp.din && !mp.feature_concat) {
        a.Wbf = p->d_packed + cp.pk_wbf;
        a.Ubf = p->d_packed + cp.pk_ubf;
        if (p->sum_variant == 8 && cp.pk_wh >= 0 && cp.pk_uh >= 0) {   // split-fp16 (DIN = H = 64)
          a.Wbf = p->d_packed + cp.pk_wh;
          a.Ubf = p->d_packed + cp.pk_uh;
          sv = 8;
        }
      }
      if (mp.aggr == IGN_AGGR_CONVOLUTION) {
        a.conv_kp = p->d_packed + p->pk_conv;
        a.conv_act = mp.act;
      }
      // the next ordered MP's input projection in the epilogue (sum_gru_g32 only)
      int target = -1, tslot = 0;
      if (b->fuse_ok && part == IGN_PART_ALL && sv == 7 && a.Wbf && a.Ubf && mp.aggr == IGN_AGGR_SUM &&
          count == mb.n_dst && mb.n_dst == b->rows[dst])
        target = fused_proj_target(p, b, mi, &tslot);
      if (target >= 0) {
        const CellP& tc = p->cells[p->mps[target].cell];
        a.proj_out = b->mp[target].d_table + b->mp[target].src_off[tslot] * 3 * tc.H;
        a.proj_W = p->d_packed + tc.pk_wbf;
        a.proj_b = p->d_packed + tc.pk_b;
        a.proj_bias_row = b->mp[target].d_table + b->mp[target].zero_row * 3 * tc.H;
      }
      const double frac = mb.n_dst ? (double)count / mb.n_dst : 0.0;
      // split GRU step (sum_gru_g32 / sum_gru_bf: x6 of x.W and h.U per 16-row tile, sum_gru_h16:
      // x3) or f32
      const bool bf = sv >= 7 && a.Wbf && a.Ubf && mp.din == cp.H && (cp.H == 32 || cp.H == 64);
      const double tiles = (double)((count + 15) / 16);
      tm.begin(K_SUM, mb.flops * frac, mb.bytes * frac,
               bf ? tiles * (sv == 8 ? 3 : 6) * 3 * (cp.H / 16) * (mp.din / 32 + cp.H / 32) * kMfmaBf16Flops : 0,
               bf ? 0 : sum_mfma_f32(count, mp.din, cp.H));
      if (pre && mb.sum_seg) {
        SumSegArgs sa{sbases.base[0], mb.d_order, mb.d_msg_ptr, mb.d_msg_src, mb.d_xsum, mb.n_seg};
        HIP_TRY(launch_sum_seg(sa, mp.din, st));
      } else if (pre) {
        SumWinArgs wa{sbases.base[0], mb.d_win_wg, mb.d_win_dst, mb.d_win_ptr, mb.d_win_src, mb.d_xsum, mb.n_win_wg};
        HIP_TRY(launch_sum_win(wa, mp.din, st));
      }
      HIP_TRY(launch_sum_gru(a, mp.din, cp.H, sv, st));
      tm.end();
      if (target >= 0) b->proj_ready[target] |= (char)(1 << tslot);
    }
  }
  if (part != IGN_PART_INTERIOR) b->cur[dst] ^= 1;   // GM:602: the destination state is overwritten
  return IGN_OK;
}

namespace {

int accumulate_stats(ign_plan* p, int n, const int* kind, const EvCost* cost);

// Resolve the pending event pairs of timed launches into the statistics (one host wait).
int flush_timing(ign_plan* p) {
  if (p->ev_slot == 0) return IGN_OK;
  const int n = p->ev_slot;
  p->ev_slot = 0;
  return accumulate_stats(p, n, p->ev_kind.data(), p->ev_cost.data());
}

// Forget the pending event pairs (the statistics are being reset).
void drop_timing(ign_plan* p) {
  if (p->ev_slot && p->stream) hipStreamSynchronize(p->stream);
  p->ev_slot = 0;
}

int accumulate_stats(ign_plan* p, int n, const int* kind, const EvCost* cost) {
  HIP_TRY(hipStreamSynchronize(p->stream));
  ign_stats_t& s = p->stats;
  s.kinds = K_KINDS;
  for (int i = 0; i < n; ++i) {
    float ms = 0;
    hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]);
    s.launches[kind[i]] += 1;
    s.ms[kind[i]] += ms;
    s.flops[kind[i]] += cost[i].flops;
    s.bytes[kind[i]] += cost[i].bytes;
    s.mfma_bf16[kind[i]] += cost[i].mfma_bf16;
    s.mfma_f32[kind[i]] += cost[i].mfma_f32;
  }
  return IGN_OK;
}

// readout launches (GM:611-629); no host synchronisation, so it can be captured
int readout(ign_plan* p, ign_batch* b) {
  hipStream_t st = p->stream;
  Timer tm{p};
  // readout (GM:611-629)
  const int64_t P = b->n_pred;
  if (!p->ro_ops.empty()) {
    tm.begin(K_OTHER, 0, 0);
    int rc = readout_ops_run(p, b, st);
    tm.end();
    if (rc) return rc;
  }
  const float* x = readout_tensor(p, b, p->ro_in[0]);
  int xs = p->ro_width;
  if (p->ro_in.size() > 1) {
    int col = 0;
    for (int id : p->ro_in) {
      const int w = p->ro_t[id].width;
      HIP_TRY(launch_concat_cols(b->d_ro_in, P, p->ro_width, col, readout_tensor(p, b, id), w, st));
      col += w;
    }
    x = b->d_ro_in;
  }
  const float* prm = p->d_params;
  if (p->fused_readout) {
    const DenseP &l1 = p->dense[0], &l2 = p->dense[1], &l3 = p->dense[2];
    Readout3Args a{x, P, xs,
                   p->d_packed + l1.pk_w, l1.use_bias ? prm + l1.off_b : nullptr,
                   p->d_packed + l2.pk_w, l2.use_bias ? prm + l2.off_b : nullptr,
                   prm + l3.off_w, l3.use_bias ? prm + l3.off_b : nullptr,
                   l1.act, l2.act, l3.act, b->d_pred};
    if (!a.b1 || !a.b2) return fail(IGN_ERR_UNSUPPORTED, "fused readout requires use_bias on hidden layers");
    double flops = 2.0 * P * ((double)l1.in * l1.out + (double)l2.in * l2.out + l3.in);
    const bool bf = p->readout_variant >= 2 && l1.pk_bf >= 0 && l2.pk_bf >= 0;
    const bool h32 = p->readout_variant == 5 && bf && l2.pk_h32 >= 0;
    const bool h16 = (p->readout_variant == 4 || (p->readout_variant == 5 && !h32)) && bf && l2.pk_h >= 0;
    const double tiles = (double)((P + 15) / 16);
    // per 16-row tile: layer 1 out/16 x in/32 and layer 2 out/16 x in/32 MFMAs of 16x16x32, x6 or x9
    // products (readout_bf); f32 (readout3): out/16 x in/4 each of 16x16x4
    const double k1 = (double)(l1.out / 16) * (l1.in / 32) + (double)(l2.out / 16) * (l2.in / 32);
    const double k1f = (double)(l1.out / 16) * (l1.in / 4) + (double)(l2.out / 16) * (l2.in / 4);
    // variant 4: both layers x3 (16x16x32 f16, the bf16 rate)
    const double kh = 3.0 * k1;
    tm.begin(K_READOUT, flops, (double)P * (4.0 * l1.in + 4.0),
             h16 || h32 ? tiles * kh * kMfmaBf16Flops : bf ? tiles * k1 * 6 * kMfmaBf16Flops : 0,
             bf ? 0 : tiles * k1f * kMfmaF32Flops);
    if (h32)   // variant 5: the same piece products on 32x32x16 (16-row-tile equivalent counted above)
      HIP_TRY(launch_readout_h32(a, p->d_packed + l2.pk_h32, l1.in, st));
    else if (h16)
      HIP_TRY(launch_readout_h16(a, p->d_packed + l2.pk_h, l1.in, st));
    else if (bf)
      HIP_TRY(launch_readout_bf(a, p->d_packed + l1.pk_bf, p->d_packed + l2.pk_bf, l1.in, 6, st));
    else
      HIP_TRY(launch_readout3(a, l1.in, l1.out, l2.out, st));
    tm.end();
  } else {
    const float* in = x;
    int in_stride = xs;
    for (size_t l = 0; l < p->dense.size(); ++l) {
      const DenseP& dl = p->dense[l];
      float* o = (l + 1 == p->dense.size()) ? b->d_pred : b->d_ro_tmp[l];
      tm.begin(K_READOUT, 2.0 * P * dl.in * dl.out, (double)P * 4.0 * (dl.in + dl.out));
      HIP_TRY(launch_dense_generic(in, P, dl.in, in_stride, prm + dl.off_w, dl.use_bias ? prm + dl.off_b : nullptr,
                                   dl.out, dl.act, o, st));
      tm.end();
      in = o;
      in_stride = dl.out;
    }
  }
  return IGN_OK;
}

int copy_out(ign_plan* p, ign_batch* b, float* pred_out) {
  if (pred_out) {
    HIP_TRY(hipMemcpyAsync(pred_out, b->d_pred, b->n_pred * b->out_units * sizeof(float), hipMemcpyDeviceToHost,
                           p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
  }
  return IGN_OK;
}

}  // namespace

// the whole MP loop of a resident batch in one launch; the final states land in
// buffer 0 of every entity, or (save: the training forward) in the state versions save names
extern "C++" int ign::resident_launch(ign_plan* p, ign_batch* b, const ResidentSave* save) {
  ResShape sh;
  if (!resident_plan_shape(p, &sh)) return fail(IGN_ERR_RUNTIME, "resident batch on a plan of another shape");
  const MPP& a = p->mps[0];
  const CellP& ca = p->cells[a.cell];
  const int path = sh.path;
  ResidentArgs r{};
  r.path_off = b->d_res_path_off;
  r.urow_off = b->d_res_urow_off;
  r.ptile_off = b->d_res_ptile_off;
  r.hdr = b->d_res_hdr;
  r.lcode_off = b->d_res_lcode_off;
  r.lcode = b->d_res_lcode;
  r.lmsg_off = b->d_res_lmsg_off;
  r.lmsg_ptr = b->d_res_lmsg_ptr;
  r.lmsg_src = b->d_res_lmsg_src;
  r.lorder = b->d_res_lorder;
  r.lnseg = b->d_res_lnseg;
  r.gorder = p->res_lpt ? b->d_res_gorder : nullptr;
  r.path_feat = b->d_feat[path];
  r.path_F = p->ents[path].feature_total;
  r.path_state = b->d_state[0][path];
  r.n_src = sh.n_src;
  for (int s = 0; s < sh.n_src; ++s) {
    const int e = sh.src_ent[s];
    const CellP& cs = p->cells[p->mps[sh.sum_mp[s]].cell];
    r.src_off[s] = b->d_res_src_off[s];
    r.src_feat[s] = b->d_feat[e];
    r.src_F[s] = p->ents[e].feature_total;
    r.src_state[s] = b->d_state[0][e];
    r.sWbf[s] = p->d_packed + cs.pk_wbf;
    r.sUbf[s] = p->d_packed + cs.pk_ubf;
    r.sum_bias[s] = p->d_packed + cs.pk_b;
  }
  r.Uh = p->d_packed + ca.pk_uh;
  r.seq_bias = p->d_packed + ca.pk_b;
  r.proj_W = p->d_packed + ca.pk_wbf;
  r.proj_b = p->d_packed + ca.pk_b;
  r.proj_Wf = p->d_packed + ca.pk_w;
  r.T = p->T;
  r.seg_on = save ? 0 : 1;   // the training forward's sums are all lane walks (sum_gru_g32 with x_save)
  if (save) {
    r.path_ver = save->path_ver;
    r.hs_save = save->hs_save;
    r.hsb = b->d_res_hsb;
    r.tab_save = save->tab_save;
    r.tab_hole = b->mp[0].zero_row;
    for (int s = 0; s < sh.n_src; ++s) r.tab_off[s] = b->mp[0].src_off[s];
    for (int s = 0; s < sh.n_src; ++s) {
      r.src_ver[s] = save->src_ver[s];
      r.x_save[s] = save->x_save[s];
    }
  }
  const ign_resident_info_t& ri = b->res_info;
  Timer tm{p};
  tm.begin(K_RESIDENT, ri.flops, ri.bytes_stage, ri.mfma_bf16, ri.mfma_f32);
  HIP_TRY(launch_resident_forward(r, b->res_graphs, save ? b->res_train_lds : b->res_lds, save ? b->res_train_form : b->res_form,
                                  save != nullptr, p->stream));
  tm.end();
  if (!save) {
    b->cur[path] = 0;
    for (int s = 0; s < sh.n_src; ++s) b->cur[sh.src_ent[s]] = 0;
  }
  return IGN_OK;
}

// IGN_RES_GROUP=K: K graphs per workgroup.  Auto (0): two where the all-LDS form of a single graph fits
// twice (NSFNET x512: 0.248-0.257 -> 0.203-0.208 ms/step, r06_c07; GEANT2's path states need the
// path-global form at two per workgroup, measured slower: 0.548 -> 0.570), else one
static int resident_batch(ign_plan* p, ign_batch* b) {
  if (p->res_group > 0) return resident_batch_k(p, b, p->res_group);
  int rc = resident_batch_k(p, b, 1);
  if (rc || !b->resident || b->res_form != IGN_RES_ALL_LDS || b->G < 2 || 2 * b->res_lds > kResidentMaxDynLds)
    return rc;
  b->resident = false;   // (the single-graph tables stay allocated until the batch goes)
  if ((rc = resident_batch_k(p, b, 2)) || b->resident) return rc;
  return resident_batch_k(p, b, 1);
}

// the batch's resident tables, built once (the first ign_forward or training forward)
extern "C++" int ign::resident_tables(ign_plan* p, ign_batch* b) {
  if (b->res_tried) return IGN_OK;
  b->res_tried = true;
  return resident_batch(p, b);
}

// MPs 1 .. S of a resident plan: the sum MP back to each source entity of MP 0 (s order)
extern "C++" int ign::resident_sum_mps(const ign_plan* p, int* sum_mp, int* n_src) {
  ResShape sh;
  if (!resident_plan_shape(p, &sh)) return 0;
  *n_src = sh.n_src;
  for (int s = 0; s < sh.n_src; ++s) sum_mp[s] = sh.sum_mp[s];
  return 1;
}

namespace {

int forward_body(ign_plan* p, ign_batch* b) {
  if (b->resident) {
    const int rc = resident_launch(p, b, nullptr);
    return rc ? rc : readout(p, b);
  }
  int rc = ign_forward_begin(p, b);
  if (rc) return rc;
  b->proj_ready.assign(p->mps.size(), 0);
  b->fuse_ok = p->fuse_proj;
  for (int it = 0; it < p->T && !rc; ++it) {            // GM:406
    b->fuse_last_iter = it + 1 == p->T;
    for (int mi = 0; mi < (int)p->mps.size() && !rc; ++mi)   // GM:410-414 (stages flattened in order)
      rc = ign_forward_mp(p, b, mi, IGN_PART_ALL);
  }
  b->fuse_ok = false;
  return rc ? rc : readout(p, b);
}

// Capture the whole forward (init, T x MPs, readout; HIP event records included when timing is
// on) into one hipGraph per batch.  The null stream cannot be captured: no graph there.
int capture(ign_plan* p, ign_batch* b) {
  if (b->graph) {
    hipGraphExecDestroy(b->graph);
    b->graph = nullptr;
  }
  if (!p->stream) return IGN_ERR_UNSUPPORTED;
  hipGraph_t g = nullptr;
  HIP_TRY(hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal));
  int rc = forward_body(p, b);
  hipError_t e = hipStreamEndCapture(p->stream, &g);
  if (rc || e != hipSuccess || !g) {
    if (g) hipGraphDestroy(g);
    hipGetLastError();
    return rc ? rc : fail(IGN_ERR_DEVICE, "hipStreamEndCapture: %s", hipGetErrorString(e));
  }
  e = hipGraphInstantiate(&b->graph, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) {
    b->graph = nullptr;
    return fail(IGN_ERR_DEVICE, "hipGraphInstantiate: %s", hipGetErrorString(e));
  }
  b->graph_timing = p->timing;
  const int n = p->timing ? p->ev_slot : 0;
  b->graph_kind.assign(p->ev_kind.begin(), p->ev_kind.begin() + n);
  b->graph_cost.assign(p->ev_cost.begin(), p->ev_cost.begin() + n);
  p->ev_slot = 0;
  return IGN_OK;
}

}  // namespace

int ign_forward_end(ign_plan* p, ign_batch* b, float* pred_out) {
  int rc = check_pb(p, b);
  if (rc) return rc;
  if ((rc = readout(p, b))) return rc;
  return copy_out(p, b, pred_out);   // timed launches stay pending until ign_stats (flush_timing)
}

int ign_forward(ign_plan* p, ign_batch* b, float* pred_out) {
  int rc = check_pb(p, b);
  if (rc) return rc;
  if ((rc = resident_tables(p, b))) return rc;   // before any capture: the tables are uploaded here
  // HIP event records captured into a graph report 0 ms on this runtime, so timed forwards
  // launch directly; untimed ones replay the captured graph
  if (p->use_graph && p->stream && !p->timing) {
    if (!b->graph) {
      if ((rc = capture(p, b))) {
        p->use_graph = false;        // not capturable here: run the launches directly from now on
        b->graph = nullptr;
        return ign_forward(p, b, pred_out);
      }
    }
    HIP_TRY(hipGraphLaunch(b->graph, p->stream));
    if ((rc = copy_out(p, b, pred_out))) return rc;
    if (p->timing)
      return accumulate_stats(p, (int)b->graph_kind.size(), b->graph_kind.data(), b->graph_cost.data());
    return IGN_OK;
  }
  if ((rc = forward_body(p, b))) return rc;
  // the event pairs stay pending (no host wait per forward, so the next forward queues behind
  // this one); ign_stats resolves them
  return copy_out(p, b, pred_out);
}

int ign_batch_read_predictions(ign_plan* p, ign_batch* b, float* host_out) {
  int rc = check_pb(p, b);
  if (rc) return rc;
  if (!host_out) return fail(IGN_ERR_INVALID, "null argument");
  return copy_out(p, b, host_out);
}

int ign_batch_mp_split(const ign_batch* b, int32_t mi, int64_t* interior, int64_t* boundary) {
  if (!b || !interior || !boundary) return fail(IGN_ERR_INVALID, "null argument");
  if (mi < 0 || mi >= (int)b->mp.size()) return fail(IGN_ERR_INVALID, "mp index %d out of range", mi);
  const MPB& mb = b->mp[mi];
  *interior = mb.sorted ? mb.n_dst : mb.n_interior;
  *boundary = mb.n_dst - *interior;
  return IGN_OK;
}

int ign_batch_bind_state(ign_plan* p, ign_batch* b, int32_t e, float* dev0, float* dev1, int64_t capacity) {
  if (!p || !b || !dev0 || !dev1) return fail(IGN_ERR_INVALID, "null argument");
  if (b->plan != p) return fail(IGN_ERR_INVALID, "batch was created for another plan");
  if (e < 0 || e >= (int)p->ents.size()) return fail(IGN_ERR_INVALID, "entity index");
  const int64_t need = (b->rows[e] + b->halo[e]) * p->ents[e].hidden_dim + 256;
  if (capacity < need) return fail(IGN_ERR_INVALID, "state buffers hold %lld floats, need %lld",
                                   (long long)capacity, (long long)need);
  if ((reinterpret_cast<uintptr_t>(dev0) | reinterpret_cast<uintptr_t>(dev1)) & 15)
    return fail(IGN_ERR_INVALID, "state buffers must be 16-byte aligned");
  b->d_state[0][e] = dev0;
  b->d_state[1][e] = dev1;
  b->cur[e] = 0;
  return IGN_OK;
}

int ign_batch_state_slot(const ign_batch* b, int32_t e, int32_t* slot) {
  if (!b || !slot) return fail(IGN_ERR_INVALID, "null argument");
  if (e < 0 || e >= (int)b->cur.size()) return fail(IGN_ERR_INVALID, "entity index");
  *slot = b->cur[e];
  return IGN_OK;
}

int ign_gather_rows(ign_plan* p, const float* src, int64_t ld, const int32_t* idx, int64_t n, int32_t cols,
                    float* dst) {
  if (!p) return fail(IGN_ERR_INVALID, "null plan");
  if (n < 0 || cols <= 0 || cols % 4 || ld < cols || ld % 4) return fail(IGN_ERR_INVALID, "gather_rows shape");
  if (n && (!src || !idx || !dst)) return fail(IGN_ERR_INVALID, "null argument");
  int rc = ensure_device(p);
  if (rc) return rc;
  HIP_TRY(launch_gather_rows(src, ld, idx, n, cols, dst, p->stream));
  return IGN_OK;
}

int ign_synchronize(ign_plan* p) {
  if (!p) return fail(IGN_ERR_INVALID, "null plan");
  int rc = ensure_device(p);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(p->stream));
  return IGN_OK;
}

int ign_batch_state(ign_plan* p, ign_batch* b, int32_t e, float* host_out) {
  if (!p || !b || !host_out) return fail(IGN_ERR_INVALID, "null argument");
  if (e < 0 || e >= (int)p->ents.size()) return fail(IGN_ERR_INVALID, "entity index");
  int rc = set_device(p->device);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(host_out, b->d_state[b->cur[e]][e], b->rows[e] * p->ents[e].hidden_dim * sizeof(float),
                         hipMemcpyDeviceToHost, p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
  return IGN_OK;
}

int ign_stats(const ign_plan* p, ign_stats_t* out) {
  if (!p || !out) return fail(IGN_ERR_INVALID, "null argument");
  int rc = flush_timing(const_cast<ign_plan*>(p));   // the plan's own bookkeeping; the ABI keeps const
  if (rc) return rc;
  *out = p->stats;
  return IGN_OK;
}

}  // extern "C"

int ign::run_message_net(ign_plan* p, const MsgNN& nn, const MPB& mb, int s, const float* src_state,
                         const float* dst_state, hipStream_t st) {
  return message_net_fwd(p, nn, mb, s, src_state, dst_state, st);
}

// Attention weights of one MP instance (AUX:287-343): per-row scores s_src = h_src (K1 a1),
// s_dst = h_dst (K2 a2), then the axis-0 softmax over (graph, position) cells into mb.d_msg_w.
int ign::attention_weights(ign_plan* p, ign_batch* b, const MPP& mp, const MPB& mb, const float* const* srcs,
                           const float* hin, hipStream_t st) {
  const CellP& cp = p->cells[mp.cell];
  const float* w12 = p->d_packed + p->pk_w12;
  for (size_t s = 0; s < mp.src.size(); ++s) {
    const int se = mp.src[s].entity;
    const int64_t rows_s = mp.nn[s].layers.empty() ? b->rows[se] + b->halo[se] : mb.n_edges[s];
    HIP_TRY(launch_dense_fwd(srcs[s], rows_s, mp.din, mp.din, nullptr, w12, nullptr, 1, IGN_ACT_LINEAR, mb.d_s_src[s],
                             st));
  }
  HIP_TRY(launch_dense_fwd(hin, mb.n_dst, cp.H, cp.H, nullptr, w12 + p->attn_F, nullptr, 1, IGN_ACT_LINEAR, mb.d_s_dst,
                           st));
  AttnArgs aa{mb.d_group_ptr, mb.d_group_empty, mb.d_cell_dst, mb.d_cell_ptr, mb.d_cell_msgs, mb.d_msg_src,
              {mb.d_s_src[0], mb.d_s_src[1], mb.d_s_src[2], mb.d_s_src[3]}, mb.d_s_dst, mb.d_ecell, mb.d_msg_w,
              mb.n_groups};
  HIP_TRY(launch_attn_softmax(aa, st));
  return IGN_OK;
}
