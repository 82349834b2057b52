// Device-side execution of collective Plans, shared by the RCCL engine (one rank per process) and
// the virtual-rank harness (N ranks in one process, device copies as the links), so the harness
// runs the production issuing code: the step / side-stream / overlap_prev event logic
// (execute_plan), the batching of a step's local ops into multi-lane launches (LocalIssuer) and
// the fp32 staging of bf16 buckets (StagedLayout). Only the transport differs:
//
//   T::coll(s, stream)        issue collective step s (RCCL collective / emulated collective)
//   T::transfers(s, stream)   issue the P2P group of step s (RCCL group / batched device copies)
//   T::has_local(s)           does step s have local reduce / copy / zero ops (on any rank)
//   T::locals(s, stream)      issue those local ops
//   T::side_stream()          the stream overlapped local ops run on
//
// Reference schedules these execute: /root/reference/src/allreduce.py:45-170 (ring, ring_gpu),
// :9-43 (central), /root/reference/src/reducers.py:38-69 (2-step node reducer).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "dla_kernels.h"
#include "plan.h"

namespace dla {
namespace comm {

#define DLA_PX_HIP(expr)                                                                                     \
  do {                                                                                                       \
    hipError_t _e = (expr);                                                                                  \
    if (_e != hipSuccess)                                                                                    \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + __FILE__ + ":" + \
                               std::to_string(__LINE__));                                                    \
  } while (0)

// Events handed out in order within one plan run and reused by the next run (a plan run records at
// most 2 events per step; every wait on them is enqueued before the next run starts).
class EventPool {
 public:
  ~EventPool() {
    for (auto e : ev_) hipEventDestroy(e);
  }
  hipEvent_t get(size_t i) {
    while (ev_.size() <= i) {
      hipEvent_t e;
      DLA_PX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ev_.push_back(e);
    }
    return ev_[i];
  }

 private:
  std::vector<hipEvent_t> ev_;
};

// Issues local ops on one stream, packing independent single-source reductions and copies into one
// multi-lane launch (launch_reduce_lanes): a ring step of C channels costs one reduce launch, not C
// (7 channels meant 7x the launches). An op that touches memory a pending lane writes,
// or writes memory a pending lane reads, flushes the batch first, so program order is preserved.
class LocalIssuer {
 public:
  LocalIssuer(int dt, size_t esz) : dt_(dt), esz_(esz) { lanes_.count = 0; }
  void set_stream(hipStream_t s) {
    if (s != st_) flush();
    st_ = s;
  }
  hipStream_t stream() const { return st_; }
  int launches() const { return launches_; }

  void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale) {
    if (n <= 0) return;
    if (nsrc <= 1) {
      add_lane(dst, nsrc ? srcs[0] : nullptr, n, scale, acc ? 1 : 0);
      return;
    }
    flush();  // k-way sums (direct / central) keep the k-source kernel: one op per step anyway
    ReduceSrcs rs{};
    rs.count = nsrc;
    for (int i = 0; i < nsrc; ++i) rs.ptr[i] = srcs[i];
    launch_reduce_sum(dst, acc, rs, n, dt_, scale, st_);
    ++launches_;
  }
  void copy(void* dst, const void* src, int64_t n) {
    if (n <= 0 || dst == src) return;
    add_lane(dst, src, n, 1.f, 2);
  }
  void zero(void* dst, int64_t n) {
    if (n <= 0) return;
    flush();
    DLA_PX_HIP(hipMemsetAsync(dst, 0, (size_t)n * esz_, st_));
    ++launches_;
  }
  void flush() {
    if (lanes_.count == 0) return;
    launch_reduce_lanes(lanes_, dt_, st_);
    ++launches_;
    lanes_.count = 0;
    w_.clear();
    r_.clear();
  }

 private:
  struct Rg {
    uintptr_t lo, hi;
  };
  static bool hit(const std::vector<Rg>& v, Rg x) {
    for (const auto& y : v)
      if (x.lo < y.hi && y.lo < x.hi) return true;
    return false;
  }
  void add_lane(void* dst, const void* src, int64_t n, float scale, int mode) {
    const Rg w{(uintptr_t)dst, (uintptr_t)dst + (uintptr_t)n * esz_};
    const Rg r{(uintptr_t)src, (uintptr_t)src + (uintptr_t)(src ? n : 0) * esz_};
    if (lanes_.count == kMaxReduceLanes || hit(w_, w) || hit(r_, w) || (src && hit(w_, r))) flush();
    ReduceLane& l = lanes_.lane[lanes_.count++];
    l.dst = dst;
    l.src = src;
    l.n = n;
    l.scale = scale;
    l.accumulate = mode;
    w_.push_back(w);
    if (src) r_.push_back(r);
  }
  int dt_;
  size_t esz_;
  hipStream_t st_ = nullptr;
  ReduceLanes lanes_;
  std::vector<Rg> w_, r_;
  int launches_ = 0;
};

inline bool is_local(const Op& o) { return o.kind == kReduce || o.kind == kCopy || o.kind == kZero; }

// Issue one rank's local ops of a step through `iss` with `ptr(Ref) -> void*`. Plans carry the
// averaging scale in their last reduces; a summing call (apply_scale false) drops it.
template <class PtrFn>
void issue_locals(const Step& step, PtrFn&& ptr, LocalIssuer& iss, bool apply_scale = true) {
  for (const auto& o : step.ops) {
    if (o.kind == kReduce) {
      const void* srcs[kPlanMaxSrc];
      for (int i = 0; i < o.nsrc; ++i) srcs[i] = ptr(o.src[i]);
      iss.reduce(ptr(o.dst), o.accumulate, srcs, o.nsrc, o.count, apply_scale ? o.scale : 1.f);
    } else if (o.kind == kCopy) {
      iss.copy(ptr(o.dst), ptr(o.src[0]), o.count);
    } else if (o.kind == kZero) {
      iss.zero(ptr(o.dst), o.count);
    }
  }
}

// Runs the step structure of a plan (`shape`: any rank's plan; all ranks share the structure) on
// stream `st`. Local ops of a step whose successor has Step::overlap_prev go to the side stream
// after an event marking the step's transfers on `st`, so they run concurrently with the
// successor's transfers; a step waits for the side work of every step before its predecessor (a
// step without the flag: of every earlier step), and `st` joins the side stream at the end.
template <class T>
void execute_plan(T& tr, const Plan& shape, hipStream_t st, EventPool& ev) {
  const size_t S = shape.steps.size();
  std::vector<hipEvent_t> side_done(S, nullptr);
  long side_last = -1, joined = -1;
  size_t nev = 0;
  auto join_upto = [&](long k) {
    for (long j = std::min(k, side_last); j > joined; --j)
      if (side_done[j]) {
        DLA_PX_HIP(hipStreamWaitEvent(st, side_done[j], 0));
        joined = j;
        break;
      }
  };
  for (size_t k = 0; k < S; ++k) {
    const Step& step = shape.steps[k];
    join_upto(step.overlap_prev ? (long)k - 2 : (long)k - 1);
    if (step.is_coll()) {
      tr.coll(k, st);
      continue;
    }
    tr.transfers(k, st);
    if (!tr.has_local(k)) continue;
    const bool side = k + 1 < S && shape.steps[k + 1].overlap_prev;
    hipStream_t ls = st;
    if (side) {
      ls = tr.side_stream();
      hipEvent_t g = ev.get(nev++);
      DLA_PX_HIP(hipEventRecord(g, st));
      DLA_PX_HIP(hipStreamWaitEvent(ls, g, 0));
    }
    tr.locals(k, ls);
    if (side) {
      side_done[k] = ev.get(nev++);
      DLA_PX_HIP(hipEventRecord(side_done[k], ls));
      side_last = (long)k;
    }
  }
  join_upto((long)S);
}

// Buffer layout of one rank's all-reduce of n elements. Without staging the plan runs on the
// bucket itself (element size of its dtype) with its scratch at `scratch`. With fp32 staging of a
// bf16 bucket the first round_up(n, 64) fp32 elements of scratch hold the staged copy the plan
// runs on, and the plan's own scratch follows.
struct StagedLayout {
  char* data;
  char* scratch;
  size_t esz;
  int dt;
};
inline size_t staged_scratch_bytes(int64_t plan_scratch_elems, int64_t n, bool staged, int dtype) {
  const size_t esz = (staged || dtype == kF32) ? 4 : 2;
  return ((size_t)plan_scratch_elems + (staged ? (size_t)((n + 63) / 64 * 64) : 0)) * esz + 512;
}
inline StagedLayout staged_layout(void* flat, int dtype, size_t esz, char* scratch, int64_t n, bool staged) {
  if (!staged) return StagedLayout{static_cast<char*>(flat), scratch, esz, dtype};
  return StagedLayout{scratch, scratch + (size_t)((n + 63) / 64 * 64) * 4, 4, kF32};
}

}  // namespace comm
}  // namespace dla
