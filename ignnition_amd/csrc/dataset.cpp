// dataset.cpp — native dataset reader: <dir>/*.tar.gz -> data.json -> the
// generator's index contract, in C++ and multi-threaded.
//
// Restates code/utils/generator_std_to_framework.py (GEN) exactly as ignnition_amd/generator.py
// does (that module is pinned bit-exact against the reference's own outputs):
//   make_indices            GEN:32-50    rank of each node within its type, `entities` key order
//   features / output       GEN:102-126  missing key -> the sample raises
//   adjacency lists         GEN:134-185  destinations in JSON key order, seq = 0..len-1 per
//                                        destination, [node, params] entries, type checks,
//                                        seq_<src>_<dst> keyed by the entity pair (the last
//                                        adjacency of a pair wins)
//   num_<entity>            GEN:188-190
//   interleave indices      GEN:193-219
//   error handling          GEN:229-230  a sample that raises abandons the rest of its file
//                                        (the error is logged); a file without data.json is fatal
// JSON objects keep their key order (the parser stores members in document order).

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "engine_internal.h"
#include "json.h"

namespace {

using ign::json::JVal;
using ign::json::JsonError;
using ign::json::Parser;

// ---------------------------------------------------------------------- tar.gz -> data.json
bool gunzip(const std::string& path, std::string& out, std::string& err) {
  gzFile f = gzopen(path.c_str(), "rb");
  if (!f) { err = "cannot open " + path; return false; }
  char buf[1 << 16];
  int n;
  while ((n = gzread(f, buf, sizeof(buf))) > 0) out.append(buf, n);
  int errnum = 0;
  const char* msg = gzerror(f, &errnum);
  gzclose(f);
  if (n < 0 || (errnum != Z_OK && errnum != Z_STREAM_END)) { err = std::string("gzip: ") + msg + " in " + path; return false; }
  return true;
}

bool tar_member(const std::string& tar, const char* name, const char** b, const char** e) {
  size_t off = 0;
  while (off + 512 <= tar.size()) {
    const char* h = tar.data() + off;
    if (h[0] == 0) break;   // end-of-archive block
    char nm[101] = {0};
    memcpy(nm, h, 100);
    char sz[13] = {0};
    memcpy(sz, h + 124, 12);
    const size_t size = strtoull(sz, nullptr, 8);
    const char type = h[156];
    std::string n(nm);
    if (n.rfind("./", 0) == 0) n = n.substr(2);
    if ((type == '0' || type == 0) && n == name) {
      if (off + 512 + size > tar.size()) return false;
      *b = h + 512;
      *e = h + 512 + size;
      return true;
    }
    off += 512 + (size + 511) / 512 * 512;
  }
  return false;
}

// ------------------------------------------------------------------------ sample -> arrays
struct Arr {
  int dtype = 0;                  // 0 float32, 1 integer (int64 values; stored narrow when they fit)
  std::vector<float> f;
  std::vector<int64_t> i;
  std::vector<int32_t> j;         // narrow: the values as int32 (i is then empty)
  bool narrow = false;
  size_t size() const { return dtype == 0 ? f.size() : narrow ? j.size() : i.size(); }
};

// a parsed sample's integer arrays (indices, counts) as int32 where every value fits: half the bytes
// a batch gather reads (a 512 x synth50 batch concatenates ~181 MB of them as int64)
void narrow_ints(Arr& a) {
  if (a.dtype != 1 || a.narrow) return;
  for (int64_t v : a.i)
    if (v < INT32_MIN || v > INT32_MAX) return;
  a.j.assign(a.i.begin(), a.i.end());
  std::vector<int64_t>().swap(a.i);
  a.narrow = true;
}

struct Sample {
  std::vector<std::pair<std::string, Arr>> kv;   // GEN dict keys in insertion order
  std::vector<float> label;
  void set(const std::string& k, Arr a) {
    for (auto& p : kv)
      if (p.first == k) { p.second = std::move(a); return; }
    kv.emplace_back(k, std::move(a));
  }
  const Arr* get(const std::string& k) const {
    for (auto& p : kv)
      if (p.first == k) return &p.second;
    return nullptr;
  }
};

struct SampleError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void flatten_numbers(const JVal& v, std::vector<float>& out) {
  if (v.t == JVal::Num || v.t == JVal::Bool) out.push_back((float)v.num);
  else if (v.t == JVal::Arr) for (auto& x : v.arr) flatten_numbers(x, out);
  else throw SampleError("a feature / label / parameter value is not numeric");
}

struct Spec {
  std::vector<std::string> features, additional;
  std::string output;
  bool training = false;
  struct Adj { std::string name, src, dst; bool params; };
  std::vector<Adj> adj;
  std::vector<std::pair<std::string, std::string>> il;   // (definition key, destination entity)
};

Sample to_data(const JVal& s, const Spec& sp) {
  if (s.t != JVal::Obj) throw SampleError("a sample is not a JSON object");
  Sample out;
  for (auto& f : sp.features) {                               // GEN:102-107
    const JVal* v = s.get(f);
    if (!v) throw SampleError("A list for feature named \"" + f + "\" was not found although being expected.");
    Arr a;
    flatten_numbers(*v, a.f);
    out.set(f, std::move(a));
  }
  for (auto& f : sp.additional) {                             // GEN:110-114
    const JVal* v = s.get(f);
    if (!v) throw SampleError("The input name \"" + f + "\" was not found although being expected.");
    Arr a;
    flatten_numbers(*v, a.f);
    out.set(f, std::move(a));
  }
  if (sp.training) {                                          // GEN:117-126
    const JVal* v = s.get(sp.output);
    if (!v) throw SampleError("A list for the output named \"" + sp.output + "\" was not found although being expected.");
    flatten_numbers(*v, out.label);
  }
  const JVal* ents = s.get("entities");                       // GEN:129-131
  if (!ents || ents->t != JVal::Obj) throw SampleError("'entities'");
  std::vector<std::pair<std::string, int64_t>> counter;       // make_indices, GEN:32-50
  std::unordered_map<std::string, std::pair<std::string, int64_t>> node;   // node -> (type, rank)
  for (auto& kv : ents->obj) {
    if (kv.second.t != JVal::Str) throw SampleError("entity type is not a string");
    const std::string& type = kv.second.str;
    auto it = std::find_if(counter.begin(), counter.end(), [&](auto& c) { return c.first == type; });
    if (it == counter.end()) { counter.emplace_back(type, 0); it = counter.end() - 1; }
    node[kv.first] = {type, it->second};                      // a repeated key keeps its last type/rank
    it->second++;
  }
  auto lookup = [&](const std::string& n) -> const std::pair<std::string, int64_t>& {
    auto it = node.find(n);
    if (it == node.end()) throw SampleError("'" + n + "'");   // KeyError in the reference
    return it->second;
  };
  std::map<std::string, std::vector<int64_t>> seq_by_pair;
  for (auto& a : sp.adj) {                                    // GEN:134-185
    const JVal* lists = s.get(a.name);
    if (!lists) throw SampleError("A list for the adjecency vector named \"" + a.name + "\" was not found although being expected.");
    if (lists->t != JVal::Obj) throw SampleError("adjacency " + a.name + " is not an object");
    Arr src, dst, seq, prm;
    src.dtype = dst.dtype = seq.dtype = 1;
    for (auto& kv : lists->obj) {
      const auto& d = lookup(kv.first);
      if (d.first != a.dst)
        throw SampleError("The adjecency list \"" + a.name + "\" was expected to be from " + a.src + " to " + a.dst +
                          ".\n However, \"" + kv.first + "\" was found which is of type \"" + d.first + "\" instead of " + a.dst);
      const JVal& sources = kv.second;
      if (sources.t != JVal::Arr) throw SampleError("adjacency sources are not a list");
      for (size_t k = 0; k < sources.arr.size(); ++k) seq.i.push_back((int64_t)k);
      if (sources.arr.empty()) throw SampleError("list index out of range");   // sources[0] on []
      if (sources.arr[0].t == JVal::Arr) {                    // [node, params] entries
        for (auto& e : sources.arr) {
          if (e.t != JVal::Arr || e.arr.empty() || e.arr[0].t != JVal::Str) throw SampleError("bad [node, params] entry");
          src.i.push_back(lookup(e.arr[0].str).second);
          dst.i.push_back(d.second);
          if (a.params) {
            if (e.arr.size() < 2) throw SampleError("list index out of range");
            flatten_numbers(e.arr[1], prm.f);
          }
        }
      } else {
        for (auto& e : sources.arr) {
          if (e.t != JVal::Str) throw SampleError("adjacency source is not a node name");
          const auto& sv = lookup(e.str);
          if (sv.first != a.src)
            throw SampleError("The adjecency list \"" + a.name + "\" was expected to be from \"" + a.src + "\" to \"" +
                              a.dst + ".\n However, \"" + kv.first + "\" was found which is of type \"" + d.first +
                              "\" instead of \"" + a.src);
          src.i.push_back(sv.second);
          dst.i.push_back(d.second);
        }
      }
    }
    const std::string sk = "seq_" + a.src + "_" + a.dst;
    seq_by_pair[sk] = seq.i;
    out.set("src_" + a.name, std::move(src));
    out.set("dst_" + a.name, std::move(dst));
    out.set(sk, std::move(seq));
    if (!prm.f.empty()) out.set("params_" + a.name, std::move(prm));
  }
  for (auto& c : counter) {                                   // GEN:188-190
    Arr n;
    n.dtype = 1;
    n.i.push_back(c.second);
    out.set("num_" + c.first, std::move(n));
  }
  for (auto& il : sp.il) {                                    // GEN:193-219
    const JVal* def = s.get(il.first);
    if (!def) throw SampleError("'" + il.first + "'");
    if (def->t != JVal::Arr) throw SampleError("interleave definition is not a list");
    std::vector<std::pair<std::string, int>> involved;
    std::vector<int> total_sequence;
    int64_t total_size = 0, n_total = 0;
    int counter_il = 0;
    for (auto& e : def->arr) {
      if (e.t != JVal::Str) throw SampleError("interleave entry is not an entity name");
      total_size += 1;
      auto it = std::find_if(involved.begin(), involved.end(), [&](auto& x) { return x.first == e.str; });
      if (it == involved.end()) {
        auto sq = seq_by_pair.find("seq_" + e.str + "_" + il.second);
        if (sq == seq_by_pair.end()) throw SampleError("'seq_" + e.str + "_" + il.second + "'");
        if (sq->second.empty()) throw SampleError("max() arg is an empty sequence");
        n_total += *std::max_element(sq->second.begin(), sq->second.end()) + 1;
        involved.emplace_back(e.str, counter_il++);
        it = involved.end() - 1;
      }
      total_sequence.push_back(it->second);
    }
    if (total_size == 0) throw SampleError("float division by zero");
    for (auto& inv : involved) {
      Arr a;
      a.dtype = 1;
      for (int64_t k = 0; k < n_total; ++k)
        if (total_sequence[k % total_size] == inv.second) a.i.push_back(k);
      out.set("indices_" + inv.first + "_to_" + il.second, std::move(a));
    }
  }
  return out;
}

// The gathered batches' concatenation buffers, recycled: a 512 x synth50 batch concatenates
// ~181 MB of int64 index lists, and writing them into fresh pages (malloc -> mmap, one page fault
// per 4 KB, serialised on the process's address-space lock when several input workers fault at
// once) costs ~3x the copy itself.  A destroyed batch hands its buffers back here (up to
// IGN_GATHER_POOL sets, default 16; each set the size of one batch); the next batch copies into
// pages that are already mapped.  Shared by the dataset and its batches, so a batch may outlive
// the dataset's handle.
struct GatherPool {
  std::mutex mu;
  std::vector<std::map<std::string, Arr>> spare;
  size_t cap = 16;
};

}  // namespace

// One gathered batch with its own buffers: any number of them may exist and be filled at once
// (one per input-pipeline worker thread); they only read the dataset's parsed samples.
struct ign_dataset_batch {
  const ign_dataset* ds = nullptr;
  std::shared_ptr<GatherPool> pool;      // null for the dataset's own `last` batch
  std::map<std::string, Arr> spare;      // recycled buffers this batch may fill, by key
  std::vector<int64_t> ids;
  std::map<std::string, Arr> cat;
  std::map<std::string, std::vector<int64_t>> lens;
  Arr labels;
  std::vector<int64_t> label_lens;
};

struct ign_dataset {
  Spec spec;
  std::vector<std::string> files;
  std::vector<std::vector<Sample>> per_file;
  std::vector<Sample*> samples;
  std::vector<std::string> errors;
  ign_dataset_batch last;   // the batch of ign_dataset_gather / ign_dataset_get
  std::shared_ptr<GatherPool> pool = std::make_shared<GatherPool>();
};

namespace {

int batch_gather(const ign_dataset* ds, ign_dataset_batch* b, const int64_t* ids, int32_t count) {
  if (!ds || !b || (!ids && count)) return fail(IGN_ERR_INVALID, "null argument");
  for (int32_t k = 0; k < count; ++k)
    if (ids[k] < 0 || ids[k] >= (int64_t)ds->samples.size()) return fail(IGN_ERR_INVALID, "sample id %lld out of range", (long long)ids[k]);
  b->ds = ds;
  b->ids.assign(ids, ids + count);
  b->cat.clear();
  b->lens.clear();
  b->labels = Arr();
  b->label_lens.clear();
  size_t n = 0;
  for (int64_t id : b->ids) n += ds->samples[id]->label.size();
  b->labels.f.reserve(n);
  for (int64_t id : b->ids) {
    const Sample& s = *ds->samples[id];
    b->labels.f.insert(b->labels.f.end(), s.label.begin(), s.label.end());
    b->label_lens.push_back((int64_t)s.label.size());
  }
  return IGN_OK;
}

// narrow: integer keys as int32 (dtype 2) when every sample's values fit, else int64 (dtype 1)
int batch_get(ign_dataset_batch* b, const char* key, int32_t* dtype, const void** ptr, int64_t* total,
              const int64_t** per_graph, bool narrow = false) {
  if (!b || !b->ds || !key || !dtype || !ptr || !total || !per_graph) return fail(IGN_ERR_INVALID, "null argument");
  std::string k(key);
  if (k == "__label__") {
    *dtype = 0;
    *ptr = b->labels.f.data();
    *total = (int64_t)b->labels.f.size();
    *per_graph = b->label_lens.data();
    return IGN_OK;
  }
  bool nw = narrow;   // every sample's array of this key stored narrow (integers only)
  if (narrow)
    for (int64_t id : b->ids) {
      const Arr* a = b->ds->samples[id]->get(k);
      if (!a || a->dtype != 1 || !a->narrow) { nw = false; break; }
    }
  const std::string ck = nw ? k + "#i32" : k;   // the concatenation's cache key
  auto it = b->cat.find(ck);
  if (it == b->cat.end()) {
    Arr c;
    auto sp = b->spare.find(ck);
    if (sp != b->spare.end()) {   // a recycled buffer: its pages are mapped already
      c = std::move(sp->second);
      b->spare.erase(sp);
      c.f.clear();
      c.i.clear();
      c.j.clear();
    }
    std::vector<int64_t> lens;
    lens.reserve(b->ids.size());
    size_t n = 0;
    for (size_t q = 0; q < b->ids.size(); ++q) {
      const int64_t id = b->ids[q];
      const Arr* a = b->ds->samples[id]->get(k);
      if (!a) return fail(IGN_ERR_INVALID, "sample %lld has no key '%s'", (long long)id, key);
      if (q == 0) c.dtype = a->dtype;
      if (a->dtype != c.dtype) return fail(IGN_ERR_INVALID, "key '%s' has mixed types", key);
      n += a->size();
    }
    c.narrow = nw;
    if (c.dtype == 0) c.f.reserve(n);
    else if (nw) c.j.reserve(n);
    else c.i.reserve(n);
    for (int64_t id : b->ids) {
      const Arr* a = b->ds->samples[id]->get(k);
      if (a->dtype == 0) c.f.insert(c.f.end(), a->f.begin(), a->f.end());
      else if (nw) c.j.insert(c.j.end(), a->j.begin(), a->j.end());
      else if (a->narrow) c.i.insert(c.i.end(), a->j.begin(), a->j.end());   // widened
      else c.i.insert(c.i.end(), a->i.begin(), a->i.end());
      lens.push_back((int64_t)a->size());
    }
    it = b->cat.emplace(ck, std::move(c)).first;
    b->lens[ck] = std::move(lens);
  }
  const Arr& c = it->second;
  *dtype = c.dtype == 0 ? 0 : c.narrow ? 2 : 1;
  *ptr = c.dtype == 0 ? (const void*)c.f.data() : c.narrow ? (const void*)c.j.data() : (const void*)c.i.data();
  *total = (int64_t)c.size();
  *per_graph = b->lens[ck].data();
  return IGN_OK;
}

}  // namespace

extern "C" {

int ign_dataset_open(const char* dir, const ign_dataset_desc* d, int32_t threads, ign_dataset** out) {
  if (!dir || !d || !out) return fail(IGN_ERR_INVALID, "null argument");
  *out = nullptr;
  std::unique_ptr<ign_dataset> ds(new ign_dataset());
  if (const char* s = getenv("IGN_GATHER_POOL")) ds->pool->cap = (size_t)std::max(0L, strtol(s, nullptr, 10));
  Spec& sp = ds->spec;
  for (int i = 0; i < d->num_features; ++i) sp.features.emplace_back(d->features[i]);
  for (int i = 0; i < d->num_additional; ++i) sp.additional.emplace_back(d->additional[i]);
  sp.training = d->output_name != nullptr;
  if (sp.training) sp.output = d->output_name;
  for (int i = 0; i < d->num_adjacencies; ++i)
    sp.adj.push_back({d->adj_name[i], d->adj_src[i], d->adj_dst[i], d->adj_params[i] != 0});
  for (int i = 0; i < d->num_interleave; ++i) sp.il.emplace_back(d->il_name[i], d->il_dst[i]);
  DIR* dh = opendir(dir);
  if (!dh) return fail(IGN_ERR_INVALID, "cannot open dataset directory %s", dir);
  while (dirent* e = readdir(dh)) {
    std::string n = e->d_name;
    if (n.size() > 7 && n.compare(n.size() - 7, 7, ".tar.gz") == 0) ds->files.push_back(std::string(dir) + "/" + n);
  }
  closedir(dh);
  std::sort(ds->files.begin(), ds->files.end());    // the Python mirror sorts the glob too
  const size_t F = ds->files.size();
  ds->per_file.resize(F);
  std::vector<std::string> ferr(F), fatal(F);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t f; (f = next.fetch_add(1)) < F;) {
      std::string tar, err;
      if (!gunzip(ds->files[f], tar, err)) { fatal[f] = err; continue; }
      const char *b = nullptr, *e = nullptr;
      if (!tar_member(tar, "data.json", &b, &e)) {   // GEN:222-223 (SystemExit)
        fatal[f] = "IGNNITION: The file data.json was not found in " + ds->files[f];
        continue;
      }
      try {
        JVal root = Parser(b, e).parse();
        if (root.t != JVal::Arr) throw JsonError("data.json is not a list of samples");
        for (auto& s : root.arr) {
          try {
            ds->per_file[f].push_back(to_data(s, sp));
            for (auto& kv : ds->per_file[f].back().kv) narrow_ints(kv.second);
          } catch (const SampleError& x) {              // GEN:229-230: log, abandon the file
            ferr[f] = x.what();
            break;
          }
        }
      } catch (const JsonError& x) {
        ferr[f] = x.what();
      }
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : 8, (int64_t)F));
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) pool.emplace_back(work);
  for (auto& t : pool) t.join();
  for (size_t f = 0; f < F; ++f)
    if (!fatal[f].empty()) return fail(IGN_ERR_INVALID, "%s", fatal[f].c_str());
  for (size_t f = 0; f < F; ++f) {
    for (auto& s : ds->per_file[f]) ds->samples.push_back(&s);
    if (!ferr[f].empty()) ds->errors.push_back("IGNNITION: " + ferr[f] + " (" + ds->files[f] + ")");
  }
  *out = ds.release();
  return IGN_OK;
}

void ign_dataset_close(ign_dataset* ds) { delete ds; }

int ign_dataset_size(const ign_dataset* ds, int64_t* n_samples, int32_t* n_errors) {
  if (!ds) return fail(IGN_ERR_INVALID, "null dataset");
  if (n_samples) *n_samples = (int64_t)ds->samples.size();
  if (n_errors) *n_errors = (int32_t)ds->errors.size();
  return IGN_OK;
}

const char* ign_dataset_error(const ign_dataset* ds, int32_t i) {
  if (!ds || i < 0 || i >= (int)ds->errors.size()) return nullptr;
  return ds->errors[i].c_str();
}

int ign_dataset_gather(ign_dataset* ds, const int64_t* ids, int32_t count) {
  if (!ds) return fail(IGN_ERR_INVALID, "null argument");
  return batch_gather(ds, &ds->last, ids, count);
}

int ign_dataset_get(ign_dataset* ds, const char* key, int32_t* dtype, const void** ptr, int64_t* total,
                    const int64_t** per_graph) {
  if (!ds) return fail(IGN_ERR_INVALID, "null argument");
  return batch_get(&ds->last, key, dtype, ptr, total, per_graph);
}

int ign_dataset_batch_create(const ign_dataset* ds, const int64_t* ids, int32_t count, ign_dataset_batch** out) {
  if (!out) return fail(IGN_ERR_INVALID, "null argument");
  *out = nullptr;
  std::unique_ptr<ign_dataset_batch> b(new ign_dataset_batch());
  if (ds) {
    b->pool = ds->pool;
    std::lock_guard<std::mutex> g(b->pool->mu);
    if (!b->pool->spare.empty()) {
      b->spare = std::move(b->pool->spare.back());
      b->pool->spare.pop_back();
    }
  }
  int rc = batch_gather(ds, b.get(), ids, count);
  if (rc) return rc;
  *out = b.release();
  return IGN_OK;
}

int ign_dataset_batch_get(ign_dataset_batch* b, const char* key, int32_t* dtype, const void** ptr, int64_t* total,
                          const int64_t** per_graph) {
  return batch_get(b, key, dtype, ptr, total, per_graph);
}

int ign_dataset_batch_get_narrow(ign_dataset_batch* b, const char* key, int32_t* dtype, const void** ptr,
                                 int64_t* total, const int64_t** per_graph) {
  return batch_get(b, key, dtype, ptr, total, per_graph, true);
}

void ign_dataset_batch_destroy(ign_dataset_batch* b) {
  if (b && b->pool) {
    std::map<std::string, Arr> keep = std::move(b->spare);
    for (auto& kv : b->cat) keep[kv.first] = std::move(kv.second);
    std::lock_guard<std::mutex> g(b->pool->mu);
    if (b->pool->spare.size() < b->pool->cap) b->pool->spare.push_back(std::move(keep));
    // else: `keep` frees its buffers when this scope ends, after the lock is released
  }
  delete b;
}

}  // extern "C"
