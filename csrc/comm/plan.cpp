// Schedule builders for the collective Plans (see plan.h).
#include "plan.h"

#include <algorithm>
#include <sstream>
#include <stdexcept>

namespace dla {
namespace comm {

namespace {

constexpr int64_t kAlign = 64;  // slice / scratch-slot alignment in elements

int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
int mod(int a, int m) { return ((a % m) + m) % m; }

void fail(const std::string& msg) { throw std::invalid_argument("comm plan: " + msg); }

void check_orders(const std::vector<std::vector<int>>& orders, int n, const char* what) {
  if (orders.empty()) fail(std::string(what) + ": no ring order");
  for (const auto& o : orders) {
    if ((int)o.size() != n) fail(std::string(what) + ": ring order must list every member once");
    std::vector<char> seen(n, 0);
    for (int v : o) {
      if (v < 0 || v >= n || seen[v]) fail(std::string(what) + ": ring order is not a permutation");
      seen[v] = 1;
    }
  }
}

Op p2p(OpKind k, int peer, Ref r, int64_t count) {
  Op o;
  o.kind = k;
  o.peer = peer;
  if (k == kSend) {
    o.src[0] = r;
    o.nsrc = 1;
  } else {
    o.dst = r;
  }
  o.count = count;
  return o;
}

Op reduce_op(Ref dst, const std::vector<Ref>& srcs, int64_t count, bool accumulate, float scale) {
  Op o;
  o.kind = kReduce;
  o.dst = dst;
  o.nsrc = (int)srcs.size();
  for (int i = 0; i < o.nsrc; ++i) o.src[i] = srcs[i];
  o.count = count;
  o.accumulate = accumulate;
  o.scale = scale;
  return o;
}

Op copy_op(Ref dst, Ref src, int64_t count) {
  Op o;
  o.kind = kCopy;
  o.dst = dst;
  o.src[0] = src;
  o.nsrc = 1;
  o.count = count;
  return o;
}

Op zero_op(Ref dst, int64_t count) {
  Op o;
  o.kind = kZero;
  o.dst = dst;
  o.count = count;
  return o;
}

Op coll_op(CollKind k, CommId comm, Ref send, Ref recv, int64_t count, bool average) {
  Op o;
  o.kind = kColl;
  o.coll = k;
  o.comm = comm;
  o.src[0] = send;
  o.nsrc = 1;
  o.dst = recv;
  o.count = count;
  o.average = average;
  return o;
}

Ref data(int64_t off) { return Ref{kData, off}; }
Ref scratch(int64_t off) { return Ref{kScratch, off}; }

// An independent region of the data buffer that one ring order walks; several lanes advance in
// lockstep (the C channels of one bucket, or the owned shards of the hierarchical inter phase).
struct Lane {
  int64_t off, len;
  std::vector<int> order;  // ring order over member indices
};

// Ring reduce-scatter over `members` (global ranks; `me` = my index). After it, the member at
// ring position p of a lane owns chunk (p + 1) % M of that lane, reduced and scaled by scale_last.
void append_ring_rs(Plan& p, const std::vector<int>& members, int me, const std::vector<Lane>& lanes,
                    float scale_last) {
  const int M = (int)members.size();
  if (M <= 1) return;
  std::vector<std::vector<int64_t>> off(lanes.size()), len(lanes.size());
  int64_t slot = 0;
  for (size_t c = 0; c < lanes.size(); ++c) {
    split(lanes[c].len, M, off[c], len[c]);
    for (auto l : len[c]) slot = std::max(slot, l);
  }
  slot = round_up(std::max<int64_t>(slot, 1), kAlign);
  p.scratch_elems = std::max(p.scratch_elems, slot * (int64_t)lanes.size());
  for (int i = 0; i < M - 1; ++i) {
    Step st, red;
    for (size_t c = 0; c < lanes.size(); ++c) {
      const auto& order = lanes[c].order;
      const int pos = (int)(std::find(order.begin(), order.end(), me) - order.begin());
      const int right = members[order[mod(pos + 1, M)]], left = members[order[mod(pos - 1, M)]];
      const int ts = mod(pos - i, M), tr = mod(ts - 1, M);
      if (len[c][ts] > 0) st.ops.push_back(p2p(kSend, right, data(lanes[c].off + off[c][ts]), len[c][ts]));
      if (len[c][tr] > 0) {
        st.ops.push_back(p2p(kRecv, left, scratch((int64_t)c * slot), len[c][tr]));
        st.ops.push_back(reduce_op(data(lanes[c].off + off[c][tr]), {scratch((int64_t)c * slot)}, len[c][tr], true,
                                   i == M - 2 ? scale_last : 1.f));
      }
    }
    // P2P ops first (one group), then the local reduces of this step
    std::stable_partition(st.ops.begin(), st.ops.end(), [](const Op& o) { return o.kind == kSend || o.kind == kRecv; });
    p.steps.push_back(std::move(st));
  }
}

// Pipelined reduce-scatter: every ring step is issued as two sub-steps, one per half of each
// lane's chunk. Sub-step (i, h) receives half h into scratch slot h of the lane and reduces it;
// the group of the next sub-step touches only the other half and the other slot, so it may overlap
// that reduce (Step::overlap_prev). A half is re-sent / its slot re-filled two sub-steps later,
// after its reduce has completed.
void append_ring_rs_pipe(Plan& p, const std::vector<int>& members, int me, const std::vector<Lane>& lanes,
                         float scale_last) {
  const int M = (int)members.size();
  if (M <= 1) return;
  const size_t C = lanes.size();
  std::vector<std::vector<int64_t>> off(C), len(C);
  int64_t slot = 0;
  for (size_t c = 0; c < C; ++c) {
    split(lanes[c].len, M, off[c], len[c]);
    for (auto l : len[c]) slot = std::max(slot, l);
  }
  slot = round_up(std::max<int64_t>((slot + 1) / 2, 1), kAlign);  // one half-chunk per slot
  p.scratch_elems = std::max(p.scratch_elems, slot * (int64_t)C * 2);
  auto half = [](int64_t l, int h, int64_t& o, int64_t& n) {
    const int64_t h0 = l > kAlign ? round_up((l + 1) / 2, kAlign) : l;  // first half 64-aligned
    o = h == 0 ? 0 : std::min(l, h0);
    n = h == 0 ? std::min(l, h0) : l - std::min(l, h0);
  };
  bool first = true;
  for (int i = 0; i < M - 1; ++i)
    for (int h = 0; h < 2; ++h) {
      Step st;
      std::vector<Op> red;
      for (size_t c = 0; c < C; ++c) {
        const auto& order = lanes[c].order;
        const int pos = (int)(std::find(order.begin(), order.end(), me) - order.begin());
        const int right = members[order[mod(pos + 1, M)]], left = members[order[mod(pos - 1, M)]];
        const int ts = mod(pos - i, M), tr = mod(ts - 1, M);
        int64_t so, sn, ro, rn;
        half(len[c][ts], h, so, sn);
        half(len[c][tr], h, ro, rn);
        const Ref sl = scratch(((int64_t)c * 2 + h) * slot);
        if (sn > 0) st.ops.push_back(p2p(kSend, right, data(lanes[c].off + off[c][ts] + so), sn));
        if (rn > 0) {
          st.ops.push_back(p2p(kRecv, left, sl, rn));
          red.push_back(reduce_op(data(lanes[c].off + off[c][tr] + ro), {sl}, rn, true, i == M - 2 ? scale_last : 1.f));
        }
      }
      for (auto& o : red) st.ops.push_back(o);
      st.overlap_prev = !first;
      first = false;
      p.steps.push_back(std::move(st));
    }
}

void append_ring_ag(Plan& p, const std::vector<int>& members, int me, const std::vector<Lane>& lanes) {
  const int M = (int)members.size();
  if (M <= 1) return;
  std::vector<std::vector<int64_t>> off(lanes.size()), len(lanes.size());
  for (size_t c = 0; c < lanes.size(); ++c) split(lanes[c].len, M, off[c], len[c]);
  for (int i = 0; i < M - 1; ++i) {
    Step st;
    for (size_t c = 0; c < lanes.size(); ++c) {
      const auto& order = lanes[c].order;
      const int pos = (int)(std::find(order.begin(), order.end(), me) - order.begin());
      const int right = members[order[mod(pos + 1, M)]], left = members[order[mod(pos - 1, M)]];
      const int ts = mod(pos - i + 1, M), tr = mod(ts - 1, M);
      if (len[c][ts] > 0) st.ops.push_back(p2p(kSend, right, data(lanes[c].off + off[c][ts]), len[c][ts]));
      if (len[c][tr] > 0) st.ops.push_back(p2p(kRecv, left, data(lanes[c].off + off[c][tr]), len[c][tr]));
    }
    p.steps.push_back(std::move(st));
  }
}

// (offset, length) this member owns in each lane after append_ring_rs.
std::vector<std::pair<int64_t, int64_t>> ring_owned(int M, int me, const std::vector<Lane>& lanes) {
  std::vector<std::pair<int64_t, int64_t>> out;
  for (const auto& l : lanes) {
    std::vector<int64_t> off, len;
    split(l.len, M, off, len);
    const int pos = (int)(std::find(l.order.begin(), l.order.end(), me) - l.order.begin());
    const int owned = mod(pos + 1, M);
    out.emplace_back(l.off + off[owned], len[owned]);
  }
  return out;
}

// Split [off, off + n) into one lane per channel order (channel c takes the c-th slice).
std::vector<Lane> channel_lanes(int64_t off, int64_t n, const std::vector<std::vector<int>>& orders) {
  // fewer channels for small buffers: every channel moves at least 4096 elements
  const int C = std::max(1, std::min<int>((int)orders.size(), (int)((n + 4095) / 4096)));
  std::vector<int64_t> co, cl;
  split(n, C, co, cl);
  std::vector<Lane> lanes;
  for (int c = 0; c < C; ++c) lanes.push_back(Lane{off + co[c], cl[c], orders[c]});
  return lanes;
}

void append_ring_allreduce(Plan& p, const std::vector<int>& members, int me, const std::vector<Lane>& lanes,
                           float scale) {
  append_ring_rs(p, members, me, lanes, scale);
  append_ring_ag(p, members, me, lanes);
}

void append_direct(Plan& p, const std::vector<int>& members, int me, int64_t base, int64_t n, float scale) {
  const int M = (int)members.size();
  if (M <= 1) return;
  std::vector<int64_t> off, len;
  split(n, M, off, len);
  int64_t maxc = 0;
  for (auto l : len) maxc = std::max(maxc, l);
  const int64_t slot = round_up(std::max<int64_t>(maxc, 1), kAlign);
  p.scratch_elems = std::max(p.scratch_elems, slot * M);
  // phase 1: my copy of chunk j goes to member j; I receive everybody's copy of my chunk
  Step s1;
  for (int k = 1; k < M; ++k) {
    const int peer = mod(me + k, M), from = mod(me - k, M);
    if (len[peer] > 0) s1.ops.push_back(p2p(kSend, members[peer], data(base + off[peer]), len[peer]));
    if (len[me] > 0) s1.ops.push_back(p2p(kRecv, members[from], scratch(slot * k), len[me]));
  }
  // one k-way reduce of my chunk in batches of kPlanMaxSrc sources (summed in k order)
  if (len[me] > 0) {
    int k = 1;
    while (k < M) {
      std::vector<Ref> srcs;
      while (k < M && (int)srcs.size() < kPlanMaxSrc) srcs.push_back(scratch(slot * k++));
      s1.ops.push_back(reduce_op(data(base + off[me]), srcs, len[me], true, k >= M ? scale : 1.f));
    }
  }
  p.steps.push_back(std::move(s1));
  // phase 2: all-gather, received in place
  Step s2;
  for (int k = 1; k < M; ++k) {
    const int peer = mod(me + k, M), from = mod(me - k, M);
    if (len[me] > 0) s2.ops.push_back(p2p(kSend, members[peer], data(base + off[me]), len[me]));
    if (len[from] > 0) s2.ops.push_back(p2p(kRecv, members[from], data(base + off[from]), len[from]));
  }
  p.steps.push_back(std::move(s2));
}

void append_central(Plan& p, const std::vector<int>& members, int me, int64_t base, int64_t n, float scale) {
  const int M = (int)members.size();
  if (M <= 1) return;
  const int64_t slot = round_up(std::max<int64_t>(n, 1), kAlign);
  Step s1, s2;
  if (me == 0) {
    p.scratch_elems = std::max(p.scratch_elems, slot * (M - 1));
    for (int r = 1; r < M; ++r) s1.ops.push_back(p2p(kRecv, members[r], scratch(slot * (r - 1)), n));
    int r = 1;
    while (r < M) {  // sum in rank order (allreduce.py:30-32)
      std::vector<Ref> srcs;
      while (r < M && (int)srcs.size() < kPlanMaxSrc) srcs.push_back(scratch(slot * (r++ - 1)));
      s1.ops.push_back(reduce_op(data(base), srcs, n, true, r >= M ? scale : 1.f));
    }
    for (int q = 1; q < M; ++q) s2.ops.push_back(p2p(kSend, members[q], data(base), n));
  } else {
    s1.ops.push_back(p2p(kSend, members[0], data(base), n));
    s2.ops.push_back(p2p(kRecv, members[0], data(base), n));
  }
  p.steps.push_back(std::move(s1));
  p.steps.push_back(std::move(s2));
}

// Central (parameter-server) all-reduce of several lanes at once: member 0 receives every member's
// copy of every lane, sums them in member order (allreduce.py:30-32) and sends the result back; two
// steps whatever the lane count.
void append_central_lanes(Plan& p, const std::vector<int>& members, int me, const std::vector<Lane>& lanes, float scale) {
  const int M = (int)members.size();
  if (M <= 1) return;
  int64_t mx = 1;
  for (const auto& l : lanes) mx = std::max(mx, l.len);
  const int64_t slot = round_up(mx, kAlign);
  Step s1, s2;
  if (me == 0) {
    p.scratch_elems = std::max(p.scratch_elems, slot * (M - 1) * (int64_t)lanes.size());
    auto at = [&](size_t c, int r) { return scratch(((int64_t)c * (M - 1) + (r - 1)) * slot); };
    for (size_t c = 0; c < lanes.size(); ++c)
      if (lanes[c].len > 0)
        for (int r = 1; r < M; ++r) s1.ops.push_back(p2p(kRecv, members[r], at(c, r), lanes[c].len));
    for (size_t c = 0; c < lanes.size(); ++c) {
      if (lanes[c].len <= 0) continue;
      int r = 1;
      while (r < M) {
        std::vector<Ref> srcs;
        while (r < M && (int)srcs.size() < kPlanMaxSrc) srcs.push_back(at(c, r++));
        s1.ops.push_back(reduce_op(data(lanes[c].off), srcs, lanes[c].len, true, r >= M ? scale : 1.f));
      }
      for (int q = 1; q < M; ++q) s2.ops.push_back(p2p(kSend, members[q], data(lanes[c].off), lanes[c].len));
    }
  } else {
    for (const auto& l : lanes)
      if (l.len > 0) {
        s1.ops.push_back(p2p(kSend, members[0], data(l.off), l.len));
        s2.ops.push_back(p2p(kRecv, members[0], data(l.off), l.len));
      }
  }
  p.steps.push_back(std::move(s1));
  p.steps.push_back(std::move(s2));
}

// ReduceScatter / (AllReduce of the shard) / AllGather on RCCL collectives. `L` members in the
// comm that reduce-scatters (kWorld for the flat algorithm, kIntra for the 2-step one), `lr` my
// index there. n not divisible by L is staged through zero-padded scratch.
void append_rs_ag_coll(Plan& p, int64_t n, int L, int lr, CommId rs_comm, bool avg_rs, int K, bool avg_inter) {
  const int64_t per = (n + L - 1) / L;
  const bool staged = per * L != n;
  auto buf = [&](int64_t off) { return staged ? scratch(off) : data(off); };
  if (staged) {
    p.scratch_elems = std::max(p.scratch_elems, per * L);
    Step s;
    s.ops.push_back(copy_op(scratch(0), data(0), n));
    s.ops.push_back(zero_op(scratch(n), per * L - n));
    p.steps.push_back(std::move(s));
  }
  if (L > 1) {
    Step s;
    s.ops.push_back(coll_op(kReduceScatter, rs_comm, buf(0), buf(per * lr), per, avg_rs));
    p.steps.push_back(std::move(s));
  }
  if (K > 1) {
    Step s;
    s.ops.push_back(coll_op(kAllReduce, kInter, buf(per * lr), buf(per * lr), per, avg_inter));
    p.steps.push_back(std::move(s));
  }
  if (L > 1) {
    Step s;
    s.ops.push_back(coll_op(kAllGather, rs_comm, buf(per * lr), buf(0), per, false));
    p.steps.push_back(std::move(s));
  }
  if (staged) {
    Step s;
    s.ops.push_back(copy_op(data(0), scratch(0), n));
    p.steps.push_back(std::move(s));
  }
}

}  // namespace

const char* algo_name(int algo) {
  switch (algo) {
    case kBuiltin: return "builtin";
    case kRing: return "ring";
    case kDirect: return "direct";
    case kCentral: return "central";
    case kRsAg: return "rsag";
    case kHierRing: return "hier_ring";
    case kHierColl: return "hier_coll";
    case kRingPipe: return "ring_pipe";
    case kHierCentral: return "hier_central";
    default: return "?";
  }
}

void split(int64_t n, int parts, std::vector<int64_t>& off, std::vector<int64_t>& len) {
  int64_t per = std::max<int64_t>(1, (n + parts - 1) / parts);
  if (per > kAlign) per = round_up(per, kAlign);
  off.resize(parts);
  len.resize(parts);
  for (int i = 0; i < parts; ++i) {
    off[i] = std::min(n, (int64_t)i * per);
    len[i] = std::max<int64_t>(0, std::min(n, off[i] + per) - off[i]);
  }
}

void Topology::validate() const {
  if (world < 1 || rank < 0 || rank >= world) fail("bad world/rank");
  const int l = L();
  if (l < 1 || world % l != 0) fail("world size is not a multiple of local_size");
  if (!rings.empty()) check_orders(rings, world, "world rings");
  if (!local_rings.empty()) check_orders(local_rings, l, "local rings");
  if (!node_rings.empty()) check_orders(node_rings, nodes(), "node rings");
}

static std::vector<std::vector<int>> identity_ring(int n) {
  std::vector<int> r(n);
  for (int i = 0; i < n; ++i) r[i] = i;
  return {r};
}

Plan build_plan(int algo, const Topology& t, int64_t n, float avg) {
  t.validate();
  Plan p;
  p.algo = algo;
  p.rank = t.rank;
  p.n = n;
  const int N = t.world;
  if (N == 1 || n == 0) return p;  // reference short-circuit (allreduce.py:18-19,55-56)
  const bool average = avg != 1.f;
  std::vector<int> world_members(N);
  for (int i = 0; i < N; ++i) world_members[i] = i;
  switch (algo) {
    case kBuiltin: {
      Step s;
      s.ops.push_back(coll_op(kAllReduce, kWorld, data(0), data(0), n, average));
      p.steps.push_back(std::move(s));
      break;
    }
    case kRsAg:
      append_rs_ag_coll(p, n, N, t.rank, kWorld, average, 1, false);
      break;
    case kRing: {
      const auto& orders = t.rings.empty() ? identity_ring(N) : t.rings;
      append_ring_allreduce(p, world_members, t.rank, channel_lanes(0, n, orders), avg);
      break;
    }
    case kRingPipe: {
      const auto& orders = t.rings.empty() ? identity_ring(N) : t.rings;
      const auto lanes = channel_lanes(0, n, orders);
      append_ring_rs_pipe(p, world_members, t.rank, lanes, avg);
      append_ring_ag(p, world_members, t.rank, lanes);  // first AG step joins every reduce
      break;
    }
    case kDirect:
      append_direct(p, world_members, t.rank, 0, n, avg);
      break;
    case kCentral:
      append_central(p, world_members, t.rank, 0, n, avg);
      break;
    case kHierRing:
    case kHierCentral: {
      const int L = t.L(), K = t.nodes();
      const int node = t.rank / L, lr = t.rank % L;
      std::vector<int> intra(L), inter(K);
      for (int j = 0; j < L; ++j) intra[j] = node * L + j;
      for (int k = 0; k < K; ++k) inter[k] = k * L + lr;
      const auto& lorders = t.local_rings.empty() ? identity_ring(L) : t.local_rings;
      const auto& norders = t.node_rings.empty() ? identity_ring(K) : t.node_rings;
      std::vector<Lane> lanes = channel_lanes(0, n, lorders);
      if (L > 1) append_ring_rs(p, intra, lr, lanes, average ? 1.f / (float)L : 1.f);
      if (K > 1) {
        std::vector<Lane> shards;
        if (L > 1) {
          auto owned = ring_owned(L, lr, lanes);
          for (size_t c = 0; c < owned.size(); ++c)
            shards.push_back(Lane{owned[c].first, owned[c].second, norders[c % norders.size()]});
        } else {
          shards = channel_lanes(0, n, norders);
        }
        if (algo == kHierCentral)
          append_central_lanes(p, inter, node, shards, average ? 1.f / (float)K : 1.f);
        else
          append_ring_allreduce(p, inter, node, shards, average ? 1.f / (float)K : 1.f);
      }
      if (L > 1) append_ring_ag(p, intra, lr, lanes);
      break;
    }
    case kHierColl: {
      const int L = t.L(), K = t.nodes();
      append_rs_ag_coll(p, n, L, t.rank % L, kIntra, average, K, average);
      break;
    }
    default:
      fail("unknown algorithm " + std::to_string(algo));
  }
  return p;
}

std::string describe(const Plan& p) {
  static const char* kinds[] = {"send", "recv", "reduce", "copy", "zero", "coll"};
  static const char* colls[] = {"allreduce", "reducescatter", "allgather"};
  static const char* comms[] = {"world", "intra", "inter"};
  auto ref = [](const Ref& r) { return std::string(r.buf == kData ? "D" : "S") + "@" + std::to_string(r.off); };
  std::ostringstream os;
  os << algo_name(p.algo) << " rank " << p.rank << " n " << p.n << " scratch " << p.scratch_elems << "\n";
  for (size_t i = 0; i < p.steps.size(); ++i) {
    os << "step " << i << (p.steps[i].overlap_prev ? " (overlaps prev local)" : "") << ":";
    for (const auto& o : p.steps[i].ops) {
      os << " [" << kinds[o.kind];
      if (o.kind == kSend) os << " ->" << o.peer << " " << ref(o.src[0]);
      if (o.kind == kRecv) os << " <-" << o.peer << " " << ref(o.dst);
      if (o.kind == kReduce) {
        os << " " << ref(o.dst) << (o.accumulate ? "+=" : "=");
        for (int s = 0; s < o.nsrc; ++s) os << (s ? "," : "") << ref(o.src[s]);
        if (o.scale != 1.f) os << " *" << o.scale;
      }
      if (o.kind == kCopy) os << " " << ref(o.dst) << "<-" << ref(o.src[0]);
      if (o.kind == kZero) os << " " << ref(o.dst);
      if (o.kind == kColl)
        os << " " << colls[o.coll] << "/" << comms[o.comm] << " " << ref(o.src[0]) << "->" << ref(o.dst)
           << (o.average ? " avg" : " sum");
      os << " x" << o.count << "]";
    }
    os << "\n";
  }
  return os.str();
}

}  // namespace comm
}  // namespace dla
