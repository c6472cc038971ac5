// Launch plan shared by the native denoiser executors (UNet, DiT).
//
// A plan is the flat list of kernel launches of one forward pass for a fixed
// batch / resolution, built once over a cached workspace and replayed on every
// call. Every pointer a launch reads is plan-owned (the caller's input and
// output are staged through plan buffers), so the whole list is captured once
// into a hipGraph and replayed with one hipGraphLaunch per forward. Profiling
// records a HIP event pair around each launch on the launch stream (on the
// observed forwards, which run launch by launch); the per-op totals are read
// back through the dm_*_profile_* ABI.
#include <cstdlib>
#pragma once
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "dm_common.h"

namespace dm {

struct Op {
  std::string label;   // kernel family / instantiation (matches the rocprof kernel name)
  double flops;        // algorithmic FLOPs of one launch
  double bytes;        // algorithmic HBM bytes of one launch (read + write of logical tensors)
  std::function<int(hipStream_t)> fn;
};

struct PlanBase {
  std::vector<void*> allocs;
  size_t bytes = 0;
  bool alloc_failed = false;
  std::vector<Op> ops;
  bool profiling = false;
  int profile_every = 1;  // record events on every N-th run only (the others run unobserved)
  long runs = 0;
  // hipGraph of the op list (captured on a private stream, launched on the caller's)
  bool graph_enabled = std::getenv("DM_NO_GRAPH") == nullptr;
  hipGraphExec_t gexec = nullptr;
  hipStream_t cap_stream = nullptr;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<double> prof_ms;
  std::vector<int64_t> prof_launches;

  PlanBase() = default;
  PlanBase(const PlanBase&) = delete;
  PlanBase& operator=(const PlanBase&) = delete;
  ~PlanBase() { release(); }

  float* alloc(size_t nbytes) {
    void* p = nullptr;
    if (hipMalloc(&p, nbytes ? nbytes : 16) != hipSuccess) {
      alloc_failed = true;
      return nullptr;
    }
    allocs.push_back(p);
    bytes += nbytes;
    return static_cast<float*>(p);
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
    for (void* a : allocs) (void)hipFree(a);
    allocs.clear();
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

}  // namespace dm
