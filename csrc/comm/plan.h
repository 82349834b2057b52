// Collective schedules as data: a Plan is the list of steps one rank executes for one all-reduce
// of `n` elements. Building the schedule is separated from running it so that
//   * the RCCL engine (engine.cpp) caches one Plan per (algorithm, bucket size) and replays it
//     every step with no per-bucket host arithmetic,
//   * the virtual-rank executor runs all N ranks' plans in lockstep inside ONE process (one GPU,
//     device copies as the links; or host memory on CPU) with exactly the production chunk
//     geometry, channel rings and reduce kernels, and checks that every send has a matching
//     receive of the same length (a schedule bug becomes an exception, not a hang).
//
// Reference schedules (/root/reference/src/allreduce.py):
//   ring     45-98   reduce-scatter + all-gather, N-1 P2P steps each, chunk (r-i)%N
//   ring_gpu 100-170 same schedule on device buffers (here: native ncclSend/ncclRecv)
//   central  9-43    root receives N-1 copies, sums in rank order, sends back
//   builtin  5-7     all_reduce(SUM) / N
// and the 2-step node reducer (/root/reference/src/reducers.py:38-69): node sum / ndevs, then the
// inter-node ring. Here it is the device hierarchy intra-node reduce-scatter -> inter-node
// all-reduce of the owned shard -> intra-node all-gather, either on P2P rings (kHierRing) or on
// RCCL collectives over ncclCommSplit sub-communicators (kHierColl).
//
// Pure host C++ (no HIP / RCCL types): unit-tested on CPU through the host executor.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace dla {
namespace comm {

enum Algo : int {
  kBuiltin = 0,   // ncclAllReduce (RCCL picks channels/protocol)
  kRing = 1,      // reference ring on ncclSend/Recv, C channels over edge-disjoint rings
  kDirect = 2,    // two-shot: P2P scatter to owners, one k-way reduce, P2P all-gather
  kCentral = 3,   // parameter server (root = rank 0)
  kRsAg = 4,      // ncclReduceScatter + ncclAllGather
  kHierRing = 5,  // 2-step on P2P rings: intra RS -> inter ring AR of owned shards -> intra AG
  kHierColl = 6,  // 2-step on sub-communicators: intra ncclReduceScatter -> inter ncclAllReduce -> intra ncclAllGather
  kRingPipe = 7,  // ring whose reduce-scatter runs in two half-chunk sub-steps: the reduce kernel of
                  // one half overlaps the P2P transfer of the other (double-buffered scratch slots)
  kHierCentral = 8,  // 2-step with a parameter server between nodes: intra RS -> the owned shards summed
                     // at node 0's rank of the same local index and sent back -> intra AG
                     // (reference main_central_reduce: NodeAgg(central), /root/reference/src/main.py:198-206)
  kAlgoCount = 9,
};
const char* algo_name(int algo);

enum BufId : uint8_t { kData = 0, kScratch = 1 };
struct Ref {
  uint8_t buf = kData;
  int64_t off = 0;  // element offset
};

enum OpKind : uint8_t { kSend, kRecv, kReduce, kCopy, kZero, kColl };
enum CollKind : uint8_t { kAllReduce, kReduceScatter, kAllGather };
enum CommId : uint8_t { kWorld = 0, kIntra = 1, kInter = 2 };

constexpr int kPlanMaxSrc = 8;  // == kMaxReduceSrc of the reduce kernel

struct Op {
  OpKind kind = kSend;
  int peer = -1;            // kSend/kRecv: global rank of the peer
  Ref dst;                  // recv / reduce / copy / zero destination; coll receive buffer
  Ref src[kPlanMaxSrc];     // send source = src[0]; reduce sources; copy source; coll send buffer
  int nsrc = 0;
  bool accumulate = false;  // reduce: dst participates in the sum
  float scale = 1.f;        // reduce: multiply the sum
  int64_t count = 0;        // elements (coll: RCCL's count argument)
  CollKind coll = kAllReduce;
  CommId comm = kWorld;
  bool average = false;     // coll: ncclAvg instead of ncclSum
};

// One step: its P2P ops (kSend/kRecv) form one RCCL group; the local ops (reduce/copy/zero) run
// after the group completed, in order. A collective step holds exactly one kColl op.
//
// overlap_prev: this step's P2P group does not touch anything the previous step's local ops read or
// write, so an executor may run those local ops concurrently with this group (RCCL engine: on a
// side stream). Local ops of every step before the previous one must have completed before the
// group starts; a step without the flag waits for all of them. The virtual-rank executor verifies
// the disjointness and executes the deferred order.
struct Step {
  std::vector<Op> ops;
  bool overlap_prev = false;
  bool is_coll() const { return ops.size() == 1 && ops[0].kind == kColl; }
};

struct Plan {
  int algo = kBuiltin;
  int rank = 0;
  int64_t n = 0;
  int64_t scratch_elems = 0;
  std::vector<Step> steps;
};

// Rank layout for building plans.
struct Topology {
  int world = 1;
  int rank = 0;
  int local_size = 0;                          // ranks per node for the 2-step algorithms (0 = world)
  std::vector<std::vector<int>> rings;         // channel ring orders over 0..world-1
  std::vector<std::vector<int>> local_rings;   // channel ring orders over 0..local_size-1
  std::vector<std::vector<int>> node_rings;    // channel ring orders over 0..num_nodes-1
  int L() const { return local_size > 0 ? local_size : world; }
  int nodes() const { return world / L(); }
  void validate() const;
};

// Elements per slice when `n` is split into `parts` contiguous slices: ceil(n / parts), rounded
// up to a multiple of 64 when it exceeds 64 (vector-aligned slice starts). Identical to the
// Python oracle's split_ranges (parallel/allreduce.py).
void split(int64_t n, int parts, std::vector<int64_t>& off, std::vector<int64_t>& len);

// The schedule rank `t.rank` executes for an all-reduce of n elements; `avg` is the final scale
// (1/world to average, 1 to sum).
Plan build_plan(int algo, const Topology& t, int64_t n, float avg);

// Human-readable dump (tests / debugging).
std::string describe(const Plan& p);

}  // namespace comm
}  // namespace dla
