// Lockstep executor for N virtual ranks inside one process.
//
// Runs the N per-rank Plans of one all-reduce step by step: at every step the P2P ops of all
// ranks are matched (the k-th send from a to b pairs with the k-th receive on b from a, the RCCL
// matching rule) and become buffer copies — the "links" — then every rank's local reduce / copy /
// zero ops run with the production reduce kernel. Collective steps (ncclAllReduce /
// ReduceScatter / AllGather on the world, intra-node or inter-node communicator) are emulated
// per communicator colour. Any schedule inconsistency — a send without a receive, mismatched
// lengths, a receive overlapping a buffer the same step sends from, ranks disagreeing on the
// step structure — throws instead of hanging, which is what a real multi-GPU run would do.
//
// The Backend supplies memory and arithmetic: the device backend (engine.cpp) issues through the
// engine's LocalIssuer (multi-lane reduce / copy launches, plan_exec.h), and the step / side-stream
// sequencing is the engine's own execute_plan driving this class's per-step calls; the host
// backend (below) runs the same arithmetic serially on CPU memory, so the schedules are checked in
// the CPU test suite too.
#pragma once

#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "plan.h"

namespace dla {
namespace comm {

template <class Backend>
class VirtualRun {
 public:
  VirtualRun(const std::vector<Plan>& plans, const Topology& topo, Backend& be) : plans_(plans), t_(topo), be_(be) {}

  // Structure checks shared by both executors: one plan per rank, same step count, collective and
  // overlap flags identical across ranks, and every overlapped step disjoint from its predecessor's
  // local ops.
  void validate() {
    const int N = (int)plans_.size();
    if (N != t_.world) fail("need one plan per virtual rank");
    const size_t S = plans_[0].steps.size();
    for (const auto& p : plans_)
      if (p.steps.size() != S) fail("ranks disagree on the number of steps");
    for (size_t s = 0; s < S; ++s) {
      const bool coll = plans_[0].steps[s].is_coll();
      const bool ovl = plans_[0].steps[s].overlap_prev;
      for (int r = 1; r < N; ++r) {
        if (plans_[r].steps[s].is_coll() != coll) fail("step " + std::to_string(s) + ": collective on some ranks only");
        if (plans_[r].steps[s].overlap_prev != ovl) fail("step " + std::to_string(s) + ": ranks disagree on overlap");
      }
      if (ovl) {
        if (coll) fail("step " + std::to_string(s) + ": a collective step cannot overlap local ops");
        if (s == 0 || plans_[0].steps[s - 1].is_coll()) fail("step " + std::to_string(s) + ": nothing to overlap");
        check_disjoint(s - 1, s);
      }
    }
  }

  // Serial executor (host backend): Step::overlap_prev defers the previous step's local ops until
  // after this step's transfers, the order a concurrent executor may produce. The device backend
  // instead runs the engine's own issuing code (plan_exec.h execute_plan) through the per-step
  // calls below.
  void run() {
    validate();
    const size_t S = plans_[0].steps.size();
    long pending = -1;
    auto flush = [&]() {
      if (pending >= 0) locals((size_t)pending);
      pending = -1;
    };
    for (size_t s = 0; s < S; ++s) {
      if (plans_[0].steps[s].is_coll()) {
        flush();
        coll(s);
        continue;
      }
      if (!plans_[0].steps[s].overlap_prev) flush();
      transfers(s);
      flush();  // the deferred local ops of step s-1 run after step s's transfers
      if (s + 1 < S && plans_[0].steps[s + 1].overlap_prev)
        pending = (long)s;
      else
        locals(s);
    }
    flush();
  }

  // ---- per-step issue (the transport interface of plan_exec.h) ----------------------------------
  bool has_local(size_t s) const {
    for (const auto& p : plans_)
      for (const Op& o : p.steps[s].ops)
        if (o.kind == kReduce || o.kind == kCopy || o.kind == kZero) return true;
    return false;
  }
  void locals(size_t s) {
    for (int r = 0; r < (int)plans_.size(); ++r)
      for (const Op& o : plans_[r].steps[s].ops) local(r, o);
  }
  void coll(size_t s) { run_coll(s); }
  void transfers(size_t s) { run_transfers(s); }

 private:
  [[noreturn]] void fail(const std::string& m) { throw std::runtime_error("virtual ranks: " + m); }

  struct Span {
    int rank;
    uint8_t buf;
    int64_t lo, hi;
  };
  static bool overlap(const Span& a, const Span& b) {
    return a.rank == b.rank && a.buf == b.buf && a.lo < b.hi && b.lo < a.hi;
  }

  // Local ops of step a vs P2P ops of step b, per rank: no write of one may meet a read or write of
  // the other.
  void check_disjoint(size_t a, size_t b) {
    for (int r = 0; r < (int)plans_.size(); ++r) {
      std::vector<Span> lw, lr, pw, pr;
      for (const Op& o : plans_[r].steps[a].ops) {
        if (o.kind == kReduce || o.kind == kCopy || o.kind == kZero) {
          lw.push_back(Span{r, o.dst.buf, o.dst.off, o.dst.off + o.count});
          if (o.kind != kZero)
            for (int i = 0; i < o.nsrc; ++i) lr.push_back(Span{r, o.src[i].buf, o.src[i].off, o.src[i].off + o.count});
        }
      }
      for (const Op& o : plans_[r].steps[b].ops) {
        if (o.kind == kSend) pr.push_back(Span{r, o.src[0].buf, o.src[0].off, o.src[0].off + o.count});
        if (o.kind == kRecv) pw.push_back(Span{r, o.dst.buf, o.dst.off, o.dst.off + o.count});
      }
      auto any = [](const std::vector<Span>& x, const std::vector<Span>& y) {
        for (const auto& u : x)
          for (const auto& v : y)
            if (overlap(u, v)) return true;
        return false;
      };
      if (any(lw, pw) || any(lw, pr) || any(lr, pw))
        fail("step " + std::to_string(b) + " overlaps the local ops of step " + std::to_string(a) + " on rank " +
             std::to_string(r) + " but touches their memory");
    }
  }

  void run_transfers(size_t s) {
    const int N = (int)plans_.size();
    std::map<std::pair<int, int>, std::deque<const Op*>> sends;  // (from, to) -> sends in issue order
    std::vector<Span> reads, writes;
    for (int r = 0; r < N; ++r)
      for (const Op& o : plans_[r].steps[s].ops) {
        if (o.kind == kSend) {
          if (o.peer < 0 || o.peer >= N || o.peer == r) fail("bad send peer");
          sends[{r, o.peer}].push_back(&o);
          reads.push_back(Span{r, o.src[0].buf, o.src[0].off, o.src[0].off + o.count});
        }
      }
    struct Xfer {
      int from, to;
      const Op *snd, *rcv;
    };
    std::vector<Xfer> xfers;
    for (int r = 0; r < N; ++r)
      for (const Op& o : plans_[r].steps[s].ops) {
        if (o.kind != kRecv) continue;
        auto it = sends.find({o.peer, r});
        if (it == sends.end() || it->second.empty())
          fail("step " + std::to_string(s) + ": rank " + std::to_string(r) + " receives from " +
               std::to_string(o.peer) + " which sends nothing");
        const Op* snd = it->second.front();
        it->second.pop_front();
        if (snd->count != o.count)
          fail("step " + std::to_string(s) + ": length mismatch " + std::to_string(o.peer) + "->" + std::to_string(r) +
               " (" + std::to_string(snd->count) + " vs " + std::to_string(o.count) + ")");
        Span w{r, o.dst.buf, o.dst.off, o.dst.off + o.count};
        for (const auto& x : writes)
          if (overlap(x, w)) fail("step " + std::to_string(s) + ": overlapping receives on rank " + std::to_string(r));
        for (const auto& x : reads)
          if (overlap(x, w))
            fail("step " + std::to_string(s) + ": rank " + std::to_string(r) + " receives into a region it sends from");
        writes.push_back(w);
        xfers.push_back(Xfer{o.peer, r, snd, &o});
      }
    for (const auto& kv : sends)
      if (!kv.second.empty())
        fail("step " + std::to_string(s) + ": send " + std::to_string(kv.first.first) + "->" +
             std::to_string(kv.first.second) + " has no matching receive");
    // the links
    for (const auto& x : xfers) be_.copy(be_.ptr(x.to, x.rcv->dst), be_.ptr(x.from, x.snd->src[0]), x.rcv->count);
  }

  void local(int r, const Op& o) {
    switch (o.kind) {
      case kReduce: {
        const void* srcs[kPlanMaxSrc];
        for (int i = 0; i < o.nsrc; ++i) srcs[i] = be_.ptr(r, o.src[i]);
        be_.reduce(be_.ptr(r, o.dst), o.accumulate, srcs, o.nsrc, o.count, o.scale);
        break;
      }
      case kCopy:
        be_.copy(be_.ptr(r, o.dst), be_.ptr(r, o.src[0]), o.count);
        break;
      case kZero:
        be_.zero(be_.ptr(r, o.dst), o.count);
        break;
      default:
        break;
    }
  }

  // members of rank r's communicator `comm`, in communicator-rank order
  std::vector<int> members(int r, CommId comm) const {
    const int N = t_.world, L = t_.L();
    std::vector<int> m;
    if (comm == kWorld) {
      for (int i = 0; i < N; ++i) m.push_back(i);
    } else if (comm == kIntra) {
      const int node = r / L;
      for (int j = 0; j < L; ++j) m.push_back(node * L + j);
    } else {
      const int lr = r % L;
      for (int k = 0; k < N / L; ++k) m.push_back(k * L + lr);
    }
    return m;
  }

  void run_coll(size_t s) {
    const int N = (int)plans_.size();
    std::vector<char> done(N, 0);
    for (int r = 0; r < N; ++r) {
      if (done[r]) continue;
      const Op& o0 = plans_[r].steps[s].ops[0];
      auto m = members(r, o0.comm);
      for (int q : m) {
        const Op& o = plans_[q].steps[s].ops[0];
        if (o.coll != o0.coll || o.comm != o0.comm || o.count != o0.count || o.average != o0.average)
          fail("step " + std::to_string(s) + ": collective arguments differ between ranks");
        done[q] = 1;
      }
      emulate(s, m, o0);
    }
  }

  // Sum `k` member buffers into `dst` (fresh), in member order, batches of kPlanMaxSrc.
  void sum_into(void* dst, const std::vector<const void*>& srcs, int64_t n, float scale) {
    size_t i = 0;
    bool first = true;
    while (i < srcs.size()) {
      const void* b[kPlanMaxSrc];
      int c = 0;
      while (i < srcs.size() && c < kPlanMaxSrc) b[c++] = srcs[i++];
      be_.reduce(dst, !first, b, c, n, i >= srcs.size() ? scale : 1.f);
      first = false;
    }
  }

  void emulate(size_t s, const std::vector<int>& m, const Op& o) {
    const int M = (int)m.size();
    const int64_t n = o.count;
    const float sc = o.average ? 1.f / (float)M : 1.f;
    auto op = [&](int j) -> const Op& { return plans_[m[j]].steps[s].ops[0]; };
    if (o.coll == kAllReduce) {
      void* tmp = be_.temp(n);
      std::vector<const void*> srcs;
      for (int j = 0; j < M; ++j) srcs.push_back(be_.ptr(m[j], op(j).src[0]));
      sum_into(tmp, srcs, n, sc);
      for (int j = 0; j < M; ++j) be_.copy(be_.ptr(m[j], op(j).dst), tmp, n);
    } else if (o.coll == kReduceScatter) {
      void* tmp = be_.temp(n * M);
      for (int j = 0; j < M; ++j) {
        std::vector<const void*> srcs;
        for (int i = 0; i < M; ++i) {
          Ref r = op(i).src[0];
          r.off += (int64_t)j * n;
          srcs.push_back(be_.ptr(m[i], r));
        }
        sum_into(be_.offset(tmp, (int64_t)j * n), srcs, n, sc);
      }
      for (int j = 0; j < M; ++j) be_.copy(be_.ptr(m[j], op(j).dst), be_.offset(tmp, (int64_t)j * n), n);
    } else {  // all-gather
      void* tmp = be_.temp(n * M);
      for (int j = 0; j < M; ++j) be_.copy(be_.offset(tmp, (int64_t)j * n), be_.ptr(m[j], op(j).src[0]), n);
      for (int i = 0; i < M; ++i) be_.copy(be_.ptr(m[i], op(i).dst), tmp, n * M);
    }
  }

  const std::vector<Plan>& plans_;
  // by value: a caller may construct the run from a temporary topology (the sanitizer build of
  // csrc/tests/host_check.cpp caught a dangling reference in exactly that use)
  const Topology t_;
  Backend& be_;
};

// Host backend: CPU buffers, fp32 or bf16 (round-to-nearest-even, as v_cvt_pk_bf16_f32). Serial:
// overlapped steps run in the deferred order (VirtualRun::run).
struct HostBackend {
  std::vector<char*> data, scratch;
  size_t esz = 4;
  bool bf16 = false;
  std::vector<std::vector<char>> temps;

  static float b2f(uint16_t v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
  }
  static uint16_t f2b(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
  }
  float load(const void* p, int64_t i) const {
    return bf16 ? b2f(static_cast<const uint16_t*>(p)[i]) : static_cast<const float*>(p)[i];
  }
  void store(void* p, int64_t i, float v) const {
    if (bf16)
      static_cast<uint16_t*>(p)[i] = f2b(v);
    else
      static_cast<float*>(p)[i] = v;
  }
  void* ptr(int rank, const Ref& r) { return (r.buf == kData ? data[rank] : scratch[rank]) + (size_t)r.off * esz; }
  void* offset(void* p, int64_t elems) { return static_cast<char*>(p) + (size_t)elems * esz; }
  void* temp(int64_t n) {
    temps.emplace_back((size_t)n * esz + 16);
    return temps.back().data();
  }
  void copy(void* dst, const void* src, int64_t n) {
    if (n > 0 && dst != src) std::memmove(dst, src, (size_t)n * esz);
  }
  void zero(void* dst, int64_t n) {
    if (n > 0) std::memset(dst, 0, (size_t)n * esz);
  }
  void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale) {
    for (int64_t i = 0; i < n; ++i) {
      float a = acc ? load(dst, i) : 0.f;
      for (int s = 0; s < nsrc; ++s) a += load(srcs[s], i);
      store(dst, i, a * scale);
    }
  }
};

}  // namespace comm
}  // namespace dla
