// IPC transport: the collective Plans of plan.h executed over peer-mapped memory instead of RCCL.
//
// Every rank owns one window (header + staged bucket + plan scratch + collective temp) whose
// IPC handle the others open once. A P2P step becomes PULLS: the receiver copies the matching
// send's source straight out of the sender's window (same device: another process's mapping of
// the same HBM; another device of the node: a load over xGMI, all peers' links at once). The
// only cross-rank synchronisation is one monotonically increasing 64-bit flag per rank, written
// solely by its owner:
//
//   P2P step s     A = ++tok: publish A ("my sends of s are produced"), wait for A from every
//                  rank I receive from; pull; B = ++tok: publish B ("I have pulled"), wait for B
//                  from every rank I send to (before I overwrite what they read).
//   AllReduce      A: all members; reduce my slice from all members' sources into my temp;
//                  C: all members (sources no longer read, temps complete); pull every slice of
//                  the result from its owner's temp; D: all members (temps no longer read).
//   ReduceScatter  A; reduce my slice from all members into temp; B; copy temp -> dst.
//   AllGather      A; pull every member's source into my dst; B.
//
// Ranks run the same step structure, so they consume tokens identically; a rank with nothing to
// do in a P2P step still advances its counter (nobody waits for it there, waits are ">=").
// Why this is correct in the plan's overlap mode (Step::overlap_prev): a peer reads my window at
// step s only where my step-s sends read, which the plan guarantees my overlapped step-(s-1)
// local ops do not write; my step-s local ops are issued after the B barrier.
//
// The runner is a template over the backend so the same protocol runs (a) on the GPU through
// the barrier kernel (ipc_sync.hip) and the engine's multi-lane copy / reduce kernels, and (b) on
// the host with one thread per rank and std::atomic flags, which is how the CPU test suite checks
// the schedule matching and the barrier protocol under real concurrency.
//
// Reference transport this replaces: Gloo isend/recv and dist.broadcast pairs
// (/root/reference/src/allreduce.py:45-170), and mp.Queue node aggregation
// (/root/reference/src/reducers.py:38-69).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "plan.h"

namespace dla {
namespace comm {

// Window header: flag u64 at 0; barrier-timeout error word (int) at 64 and its record (awaited token,
// last value seen, peer rank: u64 x3) at 72; the window's identity nonce (u64, written by the owner
// when it allocates) at 128, which every importer reads back through its mapping before first use.
constexpr size_t kIpcHeaderBytes = 4096;
constexpr size_t kIpcErrOffset = 64;
constexpr size_t kIpcDiagOffset = 72;
constexpr size_t kIpcNonceOffset = 128;

inline int64_t ipc_round64(int64_t v) { return (v + 63) / 64 * 64; }

// members of rank r's communicator `comm` (global ranks, communicator-rank order)
inline std::vector<int> comm_members(const Topology& t, int r, CommId comm) {
  const int N = t.world, L = t.L();
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

struct IpcPull {
  Ref dst;     // in my window
  int peer;    // whose window
  Ref src;     // in the peer's window
  int64_t count;
};

struct IpcStep {
  bool coll = false;
  std::vector<int> recv_from, send_to;  // P2P: distinct peers
  std::vector<IpcPull> pulls;           // P2P: in issue order
  // collective: members and each member's source / destination Ref (from its own plan)
  std::vector<int> members;
  std::vector<Ref> msrc, mdst;
  int me_idx = -1;
};

// Window layout of one all-reduce of n elements (in elements of the window's element size), the
// same on every rank: [staged data | plan scratch (max over ranks) | collective temp].
struct IpcSchedule {
  std::vector<IpcStep> steps;
  int64_t scratch_off = 0, temp_off = 0, total = 0;
  int tokens = 0;  // barrier tokens one run consumes (identical on all ranks)
};

inline IpcSchedule build_ipc_schedule(const std::vector<Plan>& plans, const Topology& t, int me, int64_t n) {
  const int N = (int)plans.size();
  if (N != t.world) throw std::runtime_error("ipc schedule: need one plan per rank");
  IpcSchedule s;
  int64_t max_scr = 0, max_tmp = 0;
  for (const auto& p : plans) max_scr = std::max(max_scr, p.scratch_elems);
  const size_t S = plans[me].steps.size();
  for (const auto& p : plans)
    if (p.steps.size() != S) throw std::runtime_error("ipc schedule: ranks disagree on the number of steps");
  for (size_t k = 0; k < S; ++k) {
    IpcStep st;
    const Step& mine = plans[me].steps[k];
    st.coll = mine.is_coll();
    for (int r = 0; r < N; ++r)
      if (plans[r].steps[k].is_coll() != st.coll)
        throw std::runtime_error("ipc schedule: step " + std::to_string(k) + " is a collective on some ranks only");
    if (st.coll) {
      const Op& o = mine.ops[0];
      st.members = comm_members(t, me, o.comm);
      for (size_t j = 0; j < st.members.size(); ++j) {
        const int q = st.members[j];
        const Op& oq = plans[q].steps[k].ops[0];
        if (oq.coll != o.coll || oq.comm != o.comm || oq.count != o.count)
          throw std::runtime_error("ipc schedule: collective arguments differ between ranks");
        st.msrc.push_back(oq.src[0]);
        st.mdst.push_back(oq.dst);
        if (q == me) st.me_idx = (int)j;
      }
      if (o.coll == kAllReduce || o.coll == kReduceScatter) max_tmp = std::max(max_tmp, o.count);
      s.tokens += o.coll == kAllReduce ? 3 : 2;
    } else {
      // the k-th receive on me from p pairs with the k-th send from p to me (RCCL matching rule)
      std::map<int, std::deque<const Op*>> sends_to_me;
      for (int p = 0; p < N; ++p) {
        if (p == me) continue;
        for (const Op& o : plans[p].steps[k].ops)
          if (o.kind == kSend && o.peer == me) sends_to_me[p].push_back(&o);
      }
      for (const Op& o : mine.ops) {
        if (o.kind == kRecv) {
          auto& q = sends_to_me[o.peer];
          if (q.empty())
            throw std::runtime_error("ipc schedule: step " + std::to_string(k) + ": receive from " +
                                     std::to_string(o.peer) + " without a matching send");
          const Op* snd = q.front();
          q.pop_front();
          if (snd->count != o.count) throw std::runtime_error("ipc schedule: send / receive length mismatch");
          st.pulls.push_back(IpcPull{o.dst, o.peer, snd->src[0], o.count});
          if (std::find(st.recv_from.begin(), st.recv_from.end(), o.peer) == st.recv_from.end())
            st.recv_from.push_back(o.peer);
        } else if (o.kind == kSend) {
          if (std::find(st.send_to.begin(), st.send_to.end(), o.peer) == st.send_to.end()) st.send_to.push_back(o.peer);
        }
      }
      for (const auto& kv : sends_to_me)
        if (!kv.second.empty()) throw std::runtime_error("ipc schedule: unmatched send to this rank");
      s.tokens += 2;
    }
    s.steps.push_back(std::move(st));
  }
  s.scratch_off = ipc_round64(n);
  s.temp_off = s.scratch_off + ipc_round64(max_scr);
  s.total = s.temp_off + ipc_round64(max_tmp);
  return s;
}

// Backend interface:
//   void* ptr(int rank, const Ref& r)       element address in rank's window (data / scratch)
//   void* tmp(int rank, int64_t off)        element address in rank's collective temp
//   void barrier(uint64_t set, const std::vector<int>& wait_ranks, uint64_t wait)
//   void copy(void* dst, const void* src, int64_t n)
//   void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale)
template <class BE>
struct IpcRunner {
  BE& be;
  const IpcSchedule& sch;
  const Plan& plan;  // this rank's
  int me;
  bool average;      // false: a summing call drops the plan's averaging
  uint64_t& tok;

  void transfers(size_t k) {
    const IpcStep& st = sch.steps[k];
    const uint64_t A = ++tok, B = ++tok;
    if (st.recv_from.empty() && st.send_to.empty()) return;
    be.barrier(A, st.recv_from, A);
    for (const auto& p : st.pulls) be.copy(be.ptr(me, p.dst), be.ptr(p.peer, p.src), p.count);
    be.barrier(B, st.send_to, B);
  }

  void coll(size_t k) {
    const IpcStep& st = sch.steps[k];
    const Op& o = plan.steps[k].ops[0];
    const int M = (int)st.members.size(), i = st.me_idx;
    std::vector<int> others;
    for (int q : st.members)
      if (q != me) others.push_back(q);
    const float sc = (o.average && average) ? 1.f / (float)M : 1.f;
    auto shifted = [](Ref r, int64_t d) {
      r.off += d;
      return r;
    };
    if (o.coll == kAllReduce) {
      const uint64_t A = ++tok, C = ++tok, D = ++tok;
      std::vector<int64_t> off, len;
      split(o.count, M, off, len);
      be.barrier(A, others, A);
      std::vector<const void*> srcs;
      for (int j = 0; j < M; ++j) srcs.push_back(be.ptr(st.members[j], shifted(st.msrc[j], off[i])));
      sum_into(be.tmp(me, off[i]), srcs, len[i], sc);
      be.barrier(C, others, C);
      for (int j = 0; j < M; ++j) be.copy(be.ptr(me, shifted(st.mdst[i], off[j])), be.tmp(st.members[j], off[j]), len[j]);
      be.barrier(D, others, D);
    } else if (o.coll == kReduceScatter) {
      const uint64_t A = ++tok, B = ++tok;
      be.barrier(A, others, A);
      std::vector<const void*> srcs;
      for (int j = 0; j < M; ++j) srcs.push_back(be.ptr(st.members[j], shifted(st.msrc[j], (int64_t)i * o.count)));
      sum_into(be.tmp(me, 0), srcs, o.count, sc);
      be.barrier(B, others, B);
      be.copy(be.ptr(me, st.mdst[i]), be.tmp(me, 0), o.count);
    } else {  // all-gather
      const uint64_t A = ++tok, B = ++tok;
      be.barrier(A, others, A);
      for (int j = 0; j < M; ++j) {
        const Ref d = shifted(st.mdst[i], (int64_t)j * o.count);
        if (j == i && d.buf == st.msrc[i].buf && d.off == st.msrc[i].off) continue;  // in place
        be.copy(be.ptr(me, d), be.ptr(st.members[j], st.msrc[j]), o.count);
      }
      be.barrier(B, others, B);
    }
  }

  // fresh sum of the sources into dst, member order, batches of kPlanMaxSrc
  void sum_into(void* dst, const std::vector<const void*>& srcs, int64_t n, float scale) {
    size_t j = 0;
    bool first = true;
    while (j < srcs.size()) {
      const void* b[kPlanMaxSrc];
      int c = 0;
      while (j < srcs.size() && c < kPlanMaxSrc) b[c++] = srcs[j++];
      be.reduce(dst, !first, b, c, n, j >= srcs.size() ? scale : 1.f);
      first = false;
    }
  }
};

// ---- host backend: one thread per rank, std::atomic flags (CPU tests of the protocol) ----------
struct IpcHostShared {
  std::vector<std::vector<char>> windows;    // element storage per rank
  std::vector<std::atomic<uint64_t>> flags;  // one per rank
  int64_t scratch_off = 0, temp_off = 0;
  size_t esz = 4;
  bool bf16 = false;
  std::atomic<double> timeout_s{30.0};
  explicit IpcHostShared(int n) : windows(n), flags(n) {
    for (auto& f : flags) f.store(0);
  }
};

struct IpcHostBackend {
  IpcHostShared& sh;
  int me;
  char* base(int r) const { return sh.windows[r].data(); }
  void* ptr(int r, const Ref& ref) const {
    return base(r) + (size_t)((ref.buf == kData ? 0 : sh.scratch_off) + ref.off) * sh.esz;
  }
  void* tmp(int r, int64_t off) const { return base(r) + (size_t)(sh.temp_off + off) * sh.esz; }
  void barrier(uint64_t set, const std::vector<int>& wait_ranks, uint64_t wait) {
    sh.flags[me].store(set, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r : wait_ranks) {
      int spins = 0;
      while (sh.flags[r].load(std::memory_order_acquire) < wait) {
        if (++spins > 256) std::this_thread::yield();
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > sh.timeout_s.load())
          throw std::runtime_error("ipc host barrier: rank " + std::to_string(r) + " never arrived (token " +
                                   std::to_string(wait) + ")");
      }
    }
  }
  static float b2f(uint16_t v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
  }
  static uint16_t f2b(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
  }
  float load(const void* p, int64_t i) const {
    return sh.bf16 ? b2f(static_cast<const uint16_t*>(p)[i]) : static_cast<const float*>(p)[i];
  }
  void store(void* p, int64_t i, float v) const {
    if (sh.bf16)
      static_cast<uint16_t*>(p)[i] = f2b(v);
    else
      static_cast<float*>(p)[i] = v;
  }
  void copy(void* dst, const void* src, int64_t n) {
    if (n > 0 && dst != src) std::memmove(dst, src, (size_t)n * sh.esz);
  }
  void zero(void* dst, int64_t n) {
    if (n > 0) std::memset(dst, 0, (size_t)n * sh.esz);
  }
  void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale) {
    for (int64_t i = 0; i < n; ++i) {
      float a = acc ? load(dst, i) : 0.f;
      for (int s = 0; s < nsrc; ++s) a += load(srcs[s], i);
      store(dst, i, a * scale);
    }
  }
};

// Run rank `me`'s plan over the host backend (serial per rank; the threads are the concurrency).
inline void ipc_host_run(IpcHostBackend& be, const IpcSchedule& sch, const Plan& plan, bool average, uint64_t& tok) {
  IpcRunner<IpcHostBackend> run{be, sch, plan, be.me, average, tok};
  for (size_t k = 0; k < plan.steps.size(); ++k) {
    const Step& st = plan.steps[k];
    if (st.is_coll()) {
      run.coll(k);
      continue;
    }
    run.transfers(k);
    for (const Op& o : st.ops) {
      if (o.kind == kReduce) {
        const void* srcs[kPlanMaxSrc];
        for (int i = 0; i < o.nsrc; ++i) srcs[i] = be.ptr(be.me, o.src[i]);
        be.reduce(be.ptr(be.me, o.dst), o.accumulate, srcs, o.nsrc, o.count, average ? o.scale : 1.f);
      } else if (o.kind == kCopy) {
        be.copy(be.ptr(be.me, o.dst), be.ptr(be.me, o.src[0]), o.count);
      } else if (o.kind == kZero) {
        be.zero(be.ptr(be.me, o.dst), o.count);
      }
    }
  }
}

}  // namespace comm
}  // namespace dla
