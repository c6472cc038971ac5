// Launch plan shared by the native denoiser executors (UNet, DiT).
//
// A plan is the flat list of kernel launches of one forward pass for a fixed
// batch / resolution, built once and replayed on every call. Every pointer a
// launch reads is plan-owned scratch (the caller's input and output are staged
// through plan buffers), so the whole list is captured once into a hipGraph and
// replayed with one hipGraphLaunch per forward. Profiling records a HIP event
// pair around each launch on the launch stream (on the observed forwards, which
// run launch by launch); the per-op totals are read back through the
// dm_*_profile_* ABI.
//
// Scratch: a plan does not own device memory. Its builder runs twice: once
// measuring (alloc hands out placeholder addresses that are never
// dereferenced, the op list is discarded), then over a ScratchPool slab large
// enough for the measured need. The plans of a model -- a small LRU cache
// keyed by the forward's shape -- and of the models that share the pool
// (dm_unet_share_workspace: UNetCombined's two networks) run over the same
// slab, since their forwards run one after the other on one stream; a plan
// that needs more than the current slab gets a larger one, and plans built
// over an older slab keep theirs until they are evicted.
#include <cstdlib>
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "dm_common.h"
#include "dm_kernels.h"

namespace dm {

struct Op {
  std::string label;   // kernel family / instantiation (matches the rocprof kernel name)
  double flops;        // algorithmic FLOPs of one launch
  double bytes;        // algorithmic HBM bytes of one launch (read + write of logical tensors)
  std::function<int(hipStream_t)> fn;
};

// One device allocation of plan scratch. Plans hold a reference to the slab they were built over, so a
// slab lives as long as some cached plan uses it.
struct Slab {
  char* base = nullptr;
  size_t bytes = 0;
  Slab() = default;
  Slab(const Slab&) = delete;
  Slab& operator=(const Slab&) = delete;
  ~Slab() {
    if (base) {
      (void)hipDeviceSynchronize();  // launches still reading the slab finish first
      (void)hipFree(base);
    }
  }
};

// The scratch of a set of plans that never run concurrently (one model's cached plans, or the models joined
// by dm_unet_share_workspace): new plans are built over the current slab; one that needs more gets a new,
// larger slab, while the plans built over the old one keep it (no rebuild) until they are evicted.
struct ScratchPool {
  std::shared_ptr<Slab> cur;
  // Stream order of the forwards over this pool's slabs: a forward on a stream other than the previous
  // forward's waits for that forward's completion event first (the slabs are shared by the cached plans and
  // by the models joined with dm_unet_share_workspace; two forwards in flight on two streams would race on
  // the scratch). Same stream: no wait, one event record per forward.
  hipEvent_t done = nullptr;
  hipStream_t last = nullptr;
  bool used = false;
  ScratchPool() = default;
  ScratchPool(const ScratchPool&) = delete;
  ScratchPool& operator=(const ScratchPool&) = delete;
  ~ScratchPool() {
    if (done) (void)hipEventDestroy(done);
  }
  int order(hipStream_t st) {
    if (used && last != st) DM_CHECK_HIP(hipStreamWaitEvent(st, done, 0));
    return DM_OK;
  }
  int mark(hipStream_t st) {
    if (!done) DM_CHECK_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    DM_CHECK_HIP(hipEventRecord(done, st));
    last = st;
    used = true;
    return DM_OK;
  }
  int ensure(size_t need, std::shared_ptr<Slab>& out) {
    if (!cur || need > cur->bytes) {
      auto s = std::make_shared<Slab>();
      void* p = nullptr;
      if (hipMalloc(&p, need ? need : 256) != hipSuccess) {
        (void)hipGetLastError();
        set_error("plan scratch allocation of " + std::to_string(need >> 20) + " MiB failed");
        return DM_ERR_HIP;
      }
      s->base = static_cast<char*>(p);
      s->bytes = need;
      cur = std::move(s);
    }
    out = cur;
    return DM_OK;
  }
  size_t bytes() const { return cur ? cur->bytes : 0; }
};

struct PlanBase {
  size_t bytes = 0;          // scratch this plan uses (offset of the bump allocator)
  bool alloc_failed = false;  // kept for the builders' checks; never set (the slab is sized beforehand)
  bool measuring = false;     // first builder pass: placeholder addresses, ops discarded
  char* scratch = nullptr;    // slab base of the real pass
  std::shared_ptr<Slab> slab;  // the slab this plan runs over (kept alive while the plan is cached)
  std::vector<Op> ops;
  bool profiling = false;
  int profile_every = 1;  // record events on every N-th run only (the others run unobserved)
  long runs = 0;
  // hipGraph of the op list (captured on a private stream, launched on the caller's)
  bool graph_enabled = true;  // Toggles::graph of the plan's build (DM_NO_GRAPH)
  Toggles toggles;            // the build's snapshot: in scope while the plan is captured or replayed op by op
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap_stream = nullptr;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<double> prof_ms;
  std::vector<int64_t> prof_launches;

  PlanBase() = default;
  PlanBase(const PlanBase&) = delete;
  PlanBase& operator=(const PlanBase&) = delete;
  virtual ~PlanBase() { release(); }

  // Bump allocation (256-B aligned) from the slab; while measuring, distinct placeholder addresses that
  // no host code dereferences (the builders write nothing into plan scratch at build time).
  float* alloc(size_t nbytes) {
    const size_t sz = ((nbytes ? nbytes : 1) + 255) & ~size_t(255);
    char* p = (measuring ? reinterpret_cast<char*>(uintptr_t(1) << 40) : scratch) + bytes;
    bytes += sz;
    return reinterpret_cast<float*>(p);
  }

  void add(std::string label, double flops, double nbytes, std::function<int(hipStream_t)> fn) {
    ops.push_back(Op{std::move(label), flops, nbytes, std::move(fn)});
  }

  void drain() {
    for (auto& e : pending) {
      float ms = 0.f;
      if (hipEventSynchronize(e.second.second) == hipSuccess &&
          hipEventElapsedTime(&ms, e.second.first, e.second.second) == hipSuccess) {
        prof_ms[e.first] += ms;
        prof_launches[e.first] += 1;
      }
      (void)hipEventDestroy(e.second.first);
      (void)hipEventDestroy(e.second.second);
    }
    pending.clear();
  }

  void invalidate_graph() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
  }

  void release() {
    drain();
    invalidate_graph();
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    cap_stream = nullptr;
  }

  int capture() {
    if (!cap_stream) DM_CHECK_HIP(hipStreamCreateWithFlags(&cap_stream, hipStreamNonBlocking));
    DM_CHECK_HIP(hipStreamBeginCapture(cap_stream, hipStreamCaptureModeThreadLocal));
    for (auto& op : ops) {
      const int rc = op.fn(cap_stream);
      if (rc) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(cap_stream, &g);
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
    }
    hipGraph_t g = nullptr;
    DM_CHECK_HIP(hipStreamEndCapture(cap_stream, &g));
    const hipError_t e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    DM_CHECK_HIP(e);
    return DM_OK;
  }

  int run(hipStream_t st) {
    ToggleScope scope(toggles);  // launch-time checks decide as the build did
    const bool observe = profiling && (runs++ % profile_every) == 0;
    if (!observe && graph_enabled) {
      if (!gexec) {
        const int rc = capture();
        if (rc) return rc;
      }
      DM_CHECK_HIP(hipGraphLaunch(gexec, st));
      return DM_OK;
    }
    for (size_t i = 0; i < ops.size(); ++i) {
      if (observe) {
        hipEvent_t a, b;
        DM_CHECK_HIP(hipEventCreate(&a));
        DM_CHECK_HIP(hipEventCreate(&b));
        DM_CHECK_HIP(hipEventRecord(a, st));
        const int rc = ops[i].fn(st);
        if (rc) return rc;
        DM_CHECK_HIP(hipEventRecord(b, st));
        pending.push_back({(int)i, {a, b}});
      } else {
        const int rc = ops[i].fn(st);
        if (rc) return rc;
      }
    }
    return DM_OK;
  }

  void profile_enable(int every) {
    drain();
    profiling = every > 0;
    profile_every = every > 0 ? every : 1;
    runs = 0;
    prof_ms.assign(ops.size(), 0.0);
    prof_launches.assign(ops.size(), 0);
  }

  int profile_get(int i, char* label, int label_len, double* flops, double* nbytes, double* ms_total,
                  int64_t* launches) {
    DM_REQUIRE(i >= 0 && i < (int)ops.size(), "op index out of range");
    drain();
    if (prof_ms.size() != ops.size()) {
      prof_ms.assign(ops.size(), 0.0);
      prof_launches.assign(ops.size(), 0);
    }
    if (label && label_len > 0) std::snprintf(label, (size_t)label_len, "%s", ops[i].label.c_str());
    if (flops) *flops = ops[i].flops;
    if (nbytes) *nbytes = ops[i].bytes;
    if (ms_total) *ms_total = prof_ms[i];
    if (launches) *launches = prof_launches[i];
    return DM_OK;
  }
};


// Small LRU of plans keyed by the forward's shape (match), all over one ScratchPool. Rebuilding a plan
// costs a synchronous build + graph capture, so alternating shapes (sample_cfg's folds, a smaller last
// fold, batched vs two-call CFG) reuse their plans instead of rebuilding on every switch.
template <class P>
struct PlanCache {
  static constexpr size_t kMaxPlans = 3;
  std::vector<std::unique_ptr<P>> plans;  // most recently used last
  std::shared_ptr<ScratchPool> pool = std::make_shared<ScratchPool>();
  long builds = 0;

  P* current() const { return plans.empty() ? nullptr : plans.back().get(); }
  void clear() { plans.clear(); }
  void invalidate_graphs() {
    for (auto& p : plans) p->invalidate_graph();
  }
  void share(const std::shared_ptr<ScratchPool>& other) {
    plans.clear();
    pool = other;
  }
  // The cached plan for which match(plan) holds, or a new one from build(plan) (called twice: measuring,
  // then over the slab).
  template <class Match, class Build>
  int get(Match match, Build build, P** out) {
    *out = nullptr;
    for (size_t i = 0; i < plans.size(); ++i) {
      if (!match(*plans[i])) continue;
      std::unique_ptr<P> p = std::move(plans[i]);
      plans.erase(plans.begin() + i);
      plans.push_back(std::move(p));
      *out = plans.back().get();
      return DM_OK;
    }
    auto m = std::make_unique<P>();
    m->measuring = true;
    int rc = build(*m);
    if (rc) return rc;
    const size_t need = m->bytes;
    m.reset();
    auto p = std::make_unique<P>();
    rc = pool->ensure(need, p->slab);
    if (rc == DM_ERR_HIP) {
      // out of device memory: drop this model's cached plans (they pin older, smaller slabs) and the pool's
      // current slab if nothing else holds it, then try once more
      plans.clear();
      if (pool->cur && pool->cur.use_count() == 1) pool->cur.reset();
      (void)hipDeviceSynchronize();
      rc = pool->ensure(need, p->slab);
    }
    if (rc) return rc;
    p->scratch = p->slab->base;
    rc = build(*p);
    if (rc) return rc;
    DM_REQUIRE(p->bytes == need, "plan builder is not deterministic (scratch size changed)");
    ++builds;
    plans.push_back(std::move(p));
    while (plans.size() > kMaxPlans) plans.erase(plans.begin());
    *out = plans.back().get();
    return DM_OK;
  }
};

}  // namespace dm
