// CommEngine: native RCCL gradient all-reduce engine (one per process group, one GPU per process),
// plus the single-process virtual-rank executor that runs the same schedules on one GPU.
//
// Replaces the reference's Python collective layer:
//   * ring_allreduce        /root/reference/src/allreduce.py:45-98   (Gloo isend/recv, CPU buffers)
//   * ring_allreduce_gpu    /root/reference/src/allreduce.py:100-170 (NCCL pairwise-broadcast emulation)
//   * central_allreduce     /root/reference/src/allreduce.py:9-43
//   * built_in_allreduce    /root/reference/src/allreduce.py:5-7
//   * ReduceImmediatelly    /root/reference/src/reducers.py:6-19 (put = reduce in the send thread)
//   * NodeAgreggateReducerCPU.pump /root/reference/src/reducers.py:38-69 (2-step, node sum + inter ring)
// and the OurDist send/receive threads (/root/reference/src/ourdist.py:102-132): instead of two
// Python threads and queues, every bucket becomes a short sequence on a dedicated high-priority
// HIP stream: wait(grad-ready event) -> [gather kernel] -> collective Plan -> record done event.
// The compute stream joins on the comm stream in sync_gradients(); the CPU never blocks on
// communication.
//
// Schedules are Plans (plan.h): built once per (algorithm, bucket size), cached, replayed. The
// engine executes a Plan's steps as RCCL groups of ncclSend/ncclRecv followed by the reduce
// kernel (reduce.hip), or as RCCL collectives on the world / intra-node / inter-node
// communicators (ncclCommSplit). VirtualComm runs the Plans of N ranks in lockstep on one GPU
// with hipMemcpyAsync as the links (vexec.h), so every algorithm's multi-rank path executes and
// is checked on a one-GPU box.
//
// Transports: RCCL (ncclSend/Recv groups and collectives), or IPC (ipc.h): each rank exports one
// window (hipIpcGetMemHandle) and the others map it; P2P steps become pulls out of the sender's
// window and collectives are emulated with the reduce kernels, ordered by per-rank flag barriers
// (ipc_sync.hip). IPC runs where RCCL cannot (several ranks on one GPU) and is a candidate
// transport on an xGMI node, where a rank's pulls load from all 7 peers at once.
//
// Failure hygiene: synchronize() polls the stream and ncclCommGetAsyncError
// with a deadline (DLA_COMM_TIMEOUT_S, default 600 s) and aborts the communicators
// (ncclCommAbort) on error or timeout instead of blocking forever; the destructor never waits
// unboundedly on a comm stream whose peer may be dead.
#include <atomic>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "dla_bindings.h"
#include "dla_kernels.h"
#include "dla_tables.h"
#include "ipc.h"
#include "plan.h"
#include "plan_exec.h"
#include "vexec.h"

namespace dla {

using comm::Plan;
using comm::Topology;

#define DLA_NCCL_CHECK(expr)                                                                  \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) {                                                                  \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")");   \
    }                                                                                         \
  } while (0)

#define DLA_HIP_THROW(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
    }                                                                                        \
  } while (0)

static ncclDataType_t nccl_dtype_of(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "CommEngine: unsupported dtype ", t);
  }
  return ncclFloat32;
}

static Topology make_topology(int rank, int world, std::vector<std::vector<int>> rings, int local_size,
                              std::vector<std::vector<int>> local_rings, std::vector<std::vector<int>> node_rings) {
  Topology t;
  t.world = world;
  t.rank = rank;
  t.local_size = (local_size <= 0 || local_size > world) ? world : local_size;
  t.rings = std::move(rings);
  t.local_rings = std::move(local_rings);
  t.node_rings = std::move(node_rings);
  try {
    t.validate();
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  return t;
}

// Algorithm codes from Python (parallel/engine.py algo_code): bits 0-3 the schedule (comm::Algo),
// bits 4-7 the ring channel count (0 = every ring of the engine's topology; a prefix of an
// edge-disjoint set is edge-disjoint), bit 8 the IPC transport (peer-mapped windows, ipc.h)
// instead of RCCL.
struct AlgoSel {
  int algo;
  int channels;
  bool ipc;
};
static AlgoSel decode_algo(int code) { return AlgoSel{code & 15, (code >> 4) & 15, ((code >> 8) & 1) != 0}; }

// Rings of `t` cut to an algorithm code's channel count (decode_algo).
static void cut_channels(Topology& t, int code) {
  const int c = decode_algo(code).channels;
  if (c > 0)
    for (auto* v : {&t.rings, &t.local_rings, &t.node_rings})
      if ((int)v->size() > c) v->resize(c);
}

// Plans are float-agnostic; these algorithms need the reduce kernel (fp32 / bf16 only). Every
// algorithm does on the IPC transport (its collectives are emulated with the reduce kernels).
static bool needs_reduce_kernel(int code) {
  const AlgoSel s = decode_algo(code);
  const int algo = s.algo;
  return s.ipc || algo == comm::kRing || algo == comm::kDirect || algo == comm::kCentral ||
         algo == comm::kHierRing || algo == comm::kRingPipe || algo == comm::kHierCentral;
}

static double comm_timeout_s() {
  const char* e = std::getenv("DLA_COMM_TIMEOUT_S");
  return e ? std::atof(e) : 600.0;
}

// ---------------------------------------------------------------------------------------------
// CommEngine
// ---------------------------------------------------------------------------------------------
class CommEngine {
 public:
  CommEngine(int rank, int world, pybind11::bytes unique_id, int device, std::vector<std::vector<int>> rings,
             int local_size, std::vector<std::vector<int>> local_rings, std::vector<std::vector<int>> node_rings)
      : device_(device),
        topo_(make_topology(rank, world, std::move(rings), local_size, std::move(local_rings), std::move(node_rings))) {
    std::string id = unique_id;
    // An empty id builds an IPC-only engine (no RCCL communicator): the ranks of a same-device
    // multi-process run, which RCCL refuses, exchange through peer-mapped windows only.
    TORCH_CHECK(id.empty() || id.size() == sizeof(ncclUniqueId), "CommEngine: bad unique id size");
    if (!id.empty()) std::memcpy(&uid_, id.data(), sizeof(ncclUniqueId));
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    // High-priority stream from torch's pool so the caching allocator knows it.
    stream_ = std::make_unique<c10::hip::HIPStream>(c10::hip::getStreamFromPool(/*isHighPriority=*/true, device_));
    int clk_khz = 100000;
    if (hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || clk_khz <= 0)
      clk_khz = 100000;
    wall_khz_ = clk_khz;
    if (!id.empty()) {
      pybind11::gil_scoped_release nogil;
      DLA_NCCL_CHECK(ncclCommInitRank(&comm_, world, uid_, rank));
      const int L = topo_.L(), K = topo_.nodes();
      // 2-step sub-communicators: ranks of one node (colour = node) and ranks with the same
      // local index on every node (colour = local index). Collective over the world comm.
      if (L > 1 && K > 1) {
        DLA_NCCL_CHECK(ncclCommSplit(comm_, rank / L, rank % L, &intra_, nullptr));
        DLA_NCCL_CHECK(ncclCommSplit(comm_, rank % L, rank / L, &inter_, nullptr));
      }
    }
    DLA_HIP_THROW(hipEventCreateWithFlags(&last_done_, hipEventDisableTiming));
  }

  ~CommEngine() {
    try {
      if (!aborted_ && comm_) {
        // bounded wait: a dead peer must not turn teardown into a hang
        if (!wait_stream(std::min(timeout_s(), 60.0), /*throw_on_fail=*/false)) abort_comms();
      }
    } catch (...) {
      abort_comms();
    }
    if (!aborted_) {
      if (inter_) ncclCommDestroy(inter_);
      if (intra_) ncclCommDestroy(intra_);
      if (comm_) ncclCommDestroy(comm_);
    }
    ipc_release();
    for (auto& e : timing_events_) hipEventDestroy(e);
    for (auto& e : ready_pool_) hipEventDestroy(e);
    if (last_done_) hipEventDestroy(last_done_);
  }

  static pybind11::bytes get_unique_id() {
    ncclUniqueId id;
    DLA_NCCL_CHECK(ncclGetUniqueId(&id));
    return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  }

  int rank() const { return topo_.rank; }
  int world() const { return topo_.world; }
  int local_size() const { return topo_.L(); }
  int num_rings() const { return (int)std::max<size_t>(1, topo_.rings.size()); }
  void set_accum_fp32(bool on) { accum_fp32_ = on; }
  // Run the whole N>1 data path (gather, fp32 staging, RCCL collective, cast back) even on one rank
  // (tests / the bench's --force_comm): at world 1 it becomes a 1-rank ncclAllReduce.
  void set_force(bool on) {
    force_ = on;
    plans_.clear();
    ipc_entries_.clear();
  }
  bool accum_fp32() const { return accum_fp32_; }

  // ---------------------------------------------------------------------------------------
  // Stream plumbing
  // ---------------------------------------------------------------------------------------
  void join_current() {
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    hipEvent_t ev = next_ready_event();
    DLA_HIP_THROW(hipEventRecord(ev, cur));
    DLA_HIP_THROW(hipStreamWaitEvent(stream_->stream(), ev, 0));
  }

  void wait_on_current() {
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    DLA_HIP_THROW(hipEventRecord(last_done_, stream_->stream()));
    DLA_HIP_THROW(hipStreamWaitEvent(cur, last_done_, 0));
  }

  // Blocks until the comm stream drained; polls RCCL's async error state and aborts the
  // communicators on error or after the deadline.
  void synchronize() {
    pybind11::gil_scoped_release nogil;
    wait_stream(timeout_s(), /*throw_on_fail=*/true);
  }

  // Current RCCL async error state of any communicator ("" = healthy).
  std::string async_error() {
    for (ncclComm_t c : {comm_, intra_, inter_}) {
      if (!c) continue;
      ncclResult_t r = ncclSuccess;
      if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
      if (r != ncclSuccess && r != ncclInProgress) return ncclGetErrorString(r);
    }
    return "";
  }

  void abort() { abort_comms(); }
  // Deadline of this engine's waits and IPC barriers (<= 0: DLA_COMM_TIMEOUT_S, default 600 s). The
  // autotuner's probe engine runs with a short one, so a candidate that hangs costs seconds and
  // aborts only the probe communicator (parallel/autotune.py).
  void set_timeout(double s) { timeout_s_ = s; }
  double timeout_s() const { return timeout_s_ > 0 ? timeout_s_ : comm_timeout_s(); }
  bool aborted() const { return aborted_; }

  uintptr_t stream_handle() const { return reinterpret_cast<uintptr_t>(stream_->stream()); }

  // Build (and cache) the plans of every bucket size up front and size the scratch buffer for the
  // largest, so no allocation ever happens mid-backward or inside a HIP-graph capture.
  // IPC codes instead record the window size they need (ipc_need); the Python front-end then
  // grows every rank's window collectively (ipc_alloc / ipc_open), since peers map it.
  void reserve(int algo, std::vector<int64_t> sizes, int dtype) {
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    if (uses_ipc(algo)) {
      for (int64_t n : sizes) {
        if ((topo_.world == 1 && !force_) || n == 0) continue;
        const size_t esz = staged(algo, dtype) ? 4 : (dtype == kBF16 ? 2 : 4);
        ipc_need_ = std::max(ipc_need_, comm::kIpcHeaderBytes + (size_t)ipc_entry(algo, n).sched.total * esz + 256);
      }
      return;
    }
    size_t need = 0;
    for (int64_t n : sizes) need = std::max(need, scratch_bytes(plan_for(algo, n), n, dtype));
    ensure_scratch(need);
  }

  // ---------------------------------------------------------------------------------------
  // IPC windows (ipc.h). Collective over the group, driven from Python: every rank calls
  // ipc_alloc(bytes) with the same size, the handles are all-gathered, every rank calls ipc_open.
  // ---------------------------------------------------------------------------------------
  bool uses_ipc(int code) const { return !comm_ || decode_algo(code).ipc; }
  int64_t ipc_need() const { return (int64_t)ipc_need_; }
  int64_t ipc_capacity() const { return (int64_t)ipc_bytes_; }
  bool has_rccl() const { return comm_ != nullptr; }
  // ranks of the RCCL communicator as RCCL itself reports them (ncclCommCount), -1 without one (IPC-only)
  int rccl_count() const {
    if (!comm_) return -1;
    int n = -1;
    DLA_NCCL_CHECK(ncclCommCount(comm_, &n));
    return n;
  }

  // Window lifecycle. A grown window is allocated while the current one (and every earlier one not
  // yet superseded by a verified mapping) stays allocated, so the new allocation can never reuse
  // the address range a peer may still hold a mapping of; the owner stamps it with `nonce`. The
  // retired windows are freed only once ipc_open has verified every peer's new mapping.
  pybind11::bytes ipc_alloc(int64_t bytes, uint64_t nonce) {
    TORCH_CHECK(bytes > (int64_t)comm::kIpcHeaderBytes, "ipc_alloc: window too small");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    drain_stream_bounded();
    void* p = nullptr;
    DLA_HIP_THROW(hipMalloc(&p, (size_t)bytes));
    // The new window stays PENDING until ipc_open has verified every peer's mapping of it: the committed
    // window (ipc_base_ / ipc_bytes_, what ipc_capacity() reports and allreduce_ipc checks against) and the
    // peer mappings change together, so a failed or stale open leaves a consistent, smaller state that the
    // next reserve grows again. An earlier pending window that never got verified is retired.
    if (ipc_pend_base_) ipc_retired_.push_back(ipc_pend_base_);
    ipc_pend_base_ = p;
    ipc_pend_bytes_ = (size_t)bytes;
    ipc_pend_nonce_ = nonce;
    DLA_HIP_THROW(hipMemset(p, 0, (size_t)bytes));
    DLA_HIP_THROW(hipMemcpy(static_cast<char*>(p) + comm::kIpcNonceOffset, &nonce, sizeof(nonce),
                            hipMemcpyHostToDevice));
    DLA_HIP_THROW(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    DLA_HIP_THROW(hipIpcGetMemHandle(&h, p));
    return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  // Map every peer's current window and read its nonce back through the mapping. Returns "" when
  // every mapping shows its owner's nonce (the previous mappings are then closed and the retired
  // windows freed); otherwise closes the new mappings, keeps the previous state and returns what
  // was wrong -- the caller (NativeEngine._map_windows) then has every rank allocate again.
  std::string ipc_open(std::vector<pybind11::bytes> handles, std::vector<uint64_t> nonces) {
    TORCH_CHECK((int)handles.size() == topo_.world && (int)nonces.size() == topo_.world,
                "ipc_open: need one handle and one nonce per rank");
    TORCH_CHECK(ipc_pend_base_, "ipc_open: call ipc_alloc first");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    std::vector<char*> fresh(topo_.world, nullptr);
    std::string bad;
    auto close_fresh = [&] {
      for (int r = 0; r < topo_.world; ++r)
        if (r != topo_.rank && fresh[r]) hipIpcCloseMemHandle(fresh[r]);
    };
    for (int r = 0; r < topo_.world; ++r) {
      if (r == topo_.rank) {
        fresh[r] = static_cast<char*>(ipc_pend_base_);
        continue;
      }
      std::string s = handles[r];
      TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "ipc_open: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, s.data(), sizeof(h));
      void* p = nullptr;
      const hipError_t oe = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
      if (oe != hipSuccess) {
        close_fresh();
        TORCH_CHECK(false, "ipc_open: hipIpcOpenMemHandle(rank ", r, "): ", hipGetErrorString(oe));
      }
      fresh[r] = static_cast<char*>(p);
      uint64_t seen = 0;
      DLA_HIP_THROW(hipMemcpy(&seen, fresh[r] + comm::kIpcNonceOffset, sizeof(seen), hipMemcpyDeviceToHost));
      if (seen != nonces[r] && bad.empty()) {
        char msg[160];
        std::snprintf(msg, sizeof(msg), "rank %d's window maps to nonce %016llx, expected %016llx", r,
                      (unsigned long long)seen, (unsigned long long)nonces[r]);
        bad = msg;
      }
    }
    if (!bad.empty()) {
      close_fresh();
      ++ipc_stale_;
      return bad;
    }
    ipc_close_peers();
    ipc_peer_ = std::move(fresh);
    if (ipc_base_) ipc_retired_.push_back(ipc_base_);
    ipc_base_ = ipc_pend_base_;
    ipc_bytes_ = ipc_pend_bytes_;
    ipc_nonce_ = ipc_pend_nonce_;
    ipc_pend_base_ = nullptr;
    ipc_pend_bytes_ = 0;
    for (void* w : ipc_retired_) hipFree(w);
    ipc_retired_.clear();
    ++ipc_generation_;
    return "";
  }

  // 1 when a barrier timed out (a peer never arrived); valid after the comm stream drained
  int ipc_error() {
    if (!ipc_base_) return 0;
    int v = 0;
    DLA_HIP_THROW(hipMemcpy(&v, static_cast<char*>(ipc_base_) + comm::kIpcErrOffset, sizeof(int), hipMemcpyDeviceToHost));
    return v;
  }

  // What the first timed-out barrier waited for: (error, awaited token, peer flag seen, peer rank,
  // host token counter, window generation, stale mappings refused so far).
  std::vector<int64_t> ipc_error_info() {
    std::vector<int64_t> out{0, 0, 0, -1, (int64_t)ipc_tok_, (int64_t)ipc_generation_, (int64_t)ipc_stale_};
    if (!ipc_base_) return out;
    uint64_t d[3] = {0, 0, 0};
    out[0] = ipc_error();
    DLA_HIP_THROW(hipMemcpy(d, static_cast<char*>(ipc_base_) + comm::kIpcDiagOffset, sizeof(d), hipMemcpyDeviceToHost));
    out[1] = (int64_t)d[0];
    out[2] = (int64_t)d[1];
    out[3] = out[0] ? (int64_t)d[2] : -1;
    return out;
  }

  // ---------------------------------------------------------------------------------------
  // Collectives. Each call enqueues onto the comm stream after joining the caller's stream.
  // ---------------------------------------------------------------------------------------
  void allreduce(at::Tensor flat, int algo, bool average) {
    check(flat);
    ++n_units_;
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    timed([&] { allreduce_on_stream(flat, algo, average, nullptr, nullptr); });
  }

  // Fused bucket path: [pack grads] -> all-reduce -> [unpack], all on the comm stream.
  // `table` is null when the gradients already live in `flat` (bucket-view mode).
  void bucket_allreduce(at::Tensor flat, int algo, bool average, PackTable* table, double pack_scale,
                        double unpack_scale) {
    check(flat);
    ++n_units_;
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    hipStream_t s = stream_->stream();
    if (table) table->pack_on(flat, pack_scale, s);
    timed([&] { allreduce_on_stream(flat, algo, average, nullptr, nullptr); });
    if (table) table->unpack_on(flat, unpack_scale, s);
  }

  // Bucket path for autograd-owned gradients: gather `grads` into `flat` at `offsets` on the comm
  // stream (by-value list launches, no per-step table upload), then all-reduce `flat` in place.
  // With accum_fp32 and a bf16 bucket the gather writes straight into the fp32 staging buffer.
  // The caller keeps `grads` alive until the compute stream has joined the comm stream.
  void bucket_allreduce_list(at::Tensor flat, int algo, bool average, std::vector<at::Tensor> grads,
                             std::vector<int64_t> offsets) {
    check(flat);
    ++n_units_;
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    timed([&] { allreduce_on_stream(flat, algo, average, &grads, &offsets); });
  }

  // Fusion-off launch group (reference main_overlap / main_onestep_overlap: one all-reduce per gradient
  // tensor, /root/reference/src/main.py:168-179,222-230): the member buckets are slices of one `group`
  // buffer at `starts` / `counts`. Every member keeps its own collective, but the group costs one event
  // join, one gather launch of all members' gradients, one fp32 staging cast and -- on the RCCL built-in
  // -- one ncclGroupStart/End around the members' ncclAllReduce calls (a single fused RCCL launch), then
  // one cast back. Other schedules / the IPC transport run the members' plans one after another after
  // the shared gather.
  void bucket_allreduce_group(at::Tensor group, std::vector<int64_t> starts, std::vector<int64_t> counts, int algo,
                              bool average, std::vector<at::Tensor> grads, std::vector<int64_t> offsets) {
    check(group);
    TORCH_CHECK(starts.size() == counts.size() && !starts.empty(), "bucket_allreduce_group: bad member spans");
    for (size_t i = 0; i < starts.size(); ++i)
      TORCH_CHECK(starts[i] >= 0 && counts[i] >= 0 && starts[i] + counts[i] <= group.numel(),
                  "bucket_allreduce_group: member ", i, " outside the group buffer");
    ++n_units_;
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    timed([&] { allreduce_group_on_stream(group, starts, counts, algo, average, grads, offsets); });
  }

  void broadcast(at::Tensor t, int root) {
    check(t);
    TORCH_CHECK(comm_, "CommEngine.broadcast needs the RCCL communicator (IPC-only engine)");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    DLA_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype_of(t.scalar_type()), root, comm_,
                                 stream_->stream()));
  }

  void allgather(at::Tensor out, at::Tensor in) {
    check(out);
    check(in);
    TORCH_CHECK(out.numel() == in.numel() * topo_.world, "allgather: out must hold world * in elements");
    TORCH_CHECK(comm_, "CommEngine.allgather needs the RCCL communicator (IPC-only engine)");
    c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
    join_current();
    pybind11::gil_scoped_release nogil;
    DLA_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype_of(in.scalar_type()), comm_,
                                 stream_->stream()));
  }

  std::string describe_plan(int algo, int64_t n) { return comm::describe(plan_for(algo, n)); }

  // Host-side issue counters: [member collectives issued (one per reduced bucket / group member, world > 1 or
  // forced), submission units (one per allreduce / bucket / group call)]; reset after reading when asked.
  std::vector<int64_t> collective_counts(bool reset) {
    std::vector<int64_t> out{n_coll_.load(), n_units_.load()};
    if (reset) {
      n_coll_ = 0;
      n_units_ = 0;
    }
    return out;
  }

  // ---------------------------------------------------------------------------------------
  // Comm-stream timing (true communication ms, SURVEY.md §7.3 hard part 6).
  // ---------------------------------------------------------------------------------------
  void set_timing(bool on) { timing_ = on; }
  double consume_comm_ms() {
    pybind11::gil_scoped_release nogil;
    double total = 0.0;
    wait_stream(timeout_s(), /*throw_on_fail=*/true);
    for (size_t i = 0; i + 1 < used_timing_; i += 2) {
      float ms = 0.f;
      DLA_HIP_THROW(hipEventElapsedTime(&ms, timing_events_[i], timing_events_[i + 1]));
      total += ms;
    }
    used_timing_ = 0;
    return total;
  }

 private:
  void check(const at::Tensor& t) {
    TORCH_CHECK(!aborted_, "CommEngine: communicator was aborted after an error");
    TORCH_CHECK(t.is_cuda() && t.device().index() == device_, "CommEngine: tensor must live on cuda:", device_);
    TORCH_CHECK(t.is_contiguous(), "CommEngine: tensor must be contiguous");
  }

  bool wait_stream(double timeout_s, bool throw_on_fail) {
    if (aborted_) {
      if (throw_on_fail) throw std::runtime_error("CommEngine: communicator was aborted after an error");
      return false;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int spins = 0;
    while (true) {
      hipError_t q = hipStreamQuery(stream_->stream());
      if (q == hipSuccess) {
        if (ipc_base_ && !ipc_broken_ && ipc_error()) {
          // the IPC windows are out of step from here on (a barrier gave up), the RCCL communicator is not:
          // refuse further IPC collectives instead of aborting RCCL
          ipc_broken_ = true;
          const std::vector<int64_t> d = ipc_error_info();
          if (throw_on_fail)
            throw std::runtime_error("CommEngine: an IPC peer did not reach a barrier within the timeout "
                                     "(DLA_COMM_TIMEOUT_S; peer failure?): waited for token " + std::to_string(d[1]) +
                                     " from rank " + std::to_string(d[3]) + ", whose flag held " + std::to_string(d[2]) +
                                     " (host counter " + std::to_string(d[4]) + ", window generation " +
                                     std::to_string(d[5]) + "); IPC transport disabled");
          return false;
        }
        return true;
      }
      if (q != hipErrorNotReady) {
        abort_comms();
        if (throw_on_fail) throw std::runtime_error(std::string("CommEngine: comm stream failed: ") + hipGetErrorString(q));
        return false;
      }
      std::string err = async_error();
      if (!err.empty()) {
        abort_comms();
        if (throw_on_fail) throw std::runtime_error("CommEngine: RCCL async error: " + err + " (communicators aborted)");
        return false;
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) {
        abort_comms();
        if (throw_on_fail)
          throw std::runtime_error("CommEngine: communication did not complete within " + std::to_string(timeout_s) +
                                   " s (peer failure?); communicators aborted");
        return false;
      }
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins > 4096 ? 1000 : 20));
    }
  }

  void ipc_close_peers() {
    for (int r = 0; r < (int)ipc_peer_.size(); ++r)
      if (r != topo_.rank && ipc_peer_[r]) hipIpcCloseMemHandle(ipc_peer_[r]);
    ipc_peer_.clear();
  }

  void drain_stream_bounded() {
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = std::min(60.0, timeout_s());
    while (hipStreamQuery(stream_->stream()) == hipErrorNotReady &&
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < limit)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
  }

  // bounded drain of the comm stream, then unmap the peers and free the windows
  void ipc_release() {
    if (!ipc_base_ && !ipc_pend_base_ && ipc_peer_.empty() && ipc_retired_.empty()) return;
    drain_stream_bounded();
    ipc_close_peers();
    for (void* w : ipc_retired_) hipFree(w);
    ipc_retired_.clear();
    if (ipc_base_) hipFree(ipc_base_);
    if (ipc_pend_base_) hipFree(ipc_pend_base_);
    ipc_base_ = ipc_pend_base_ = nullptr;
    ipc_bytes_ = ipc_pend_bytes_ = 0;
  }

  void abort_comms() {
    if (aborted_) return;
    aborted_ = true;
    if (inter_) ncclCommAbort(inter_);
    if (intra_) ncclCommAbort(intra_);
    if (comm_) ncclCommAbort(comm_);
  }

  hipEvent_t next_ready_event() {
    // Events are recycled round-robin; a pool of 512 is far more than the buckets in flight.
    if (ready_pool_.size() < 512) {
      hipEvent_t e;
      DLA_HIP_THROW(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ready_pool_.push_back(e);
      return e;
    }
    hipEvent_t e = ready_pool_[ready_next_];
    ready_next_ = (ready_next_ + 1) % ready_pool_.size();
    return e;
  }

  template <typename F>
  void timed(F&& f) {
    if (!timing_) {
      f();
      return;
    }
    while (timing_events_.size() < used_timing_ + 2) {
      hipEvent_t e;
      DLA_HIP_THROW(hipEventCreate(&e));
      timing_events_.push_back(e);
    }
    DLA_HIP_THROW(hipEventRecord(timing_events_[used_timing_], stream_->stream()));
    f();
    DLA_HIP_THROW(hipEventRecord(timing_events_[used_timing_ + 1], stream_->stream()));
    used_timing_ += 2;
  }

  // the engine's topology seen from `rank`, its rings cut to the code's channel count
  Topology topo_for(int code, int rank) const {
    Topology t = topo_;
    t.rank = rank;
    cut_channels(t, code);
    return t;
  }

  const Plan& plan_for(int code, int64_t n) {
    auto key = std::make_pair(code, n);
    auto it = plans_.find(key);
    if (it != plans_.end()) return it->second;
    return plans_.emplace(key, make_plan(code, topo_.rank, n)).first->second;
  }

  struct IpcEntry {
    std::vector<Plan> plans;  // every rank's (the receiver matches its pulls against the senders')
    comm::IpcSchedule sched;
  };

  const IpcEntry& ipc_entry(int code, int64_t n) {
    auto key = std::make_pair(code, n);
    auto it = ipc_entries_.find(key);
    if (it != ipc_entries_.end()) return it->second;
    IpcEntry e;
    for (int r = 0; r < topo_.world; ++r) e.plans.push_back(make_plan(code, r, n));
    try {
      e.sched = comm::build_ipc_schedule(e.plans, topo_for(code, topo_.rank), topo_.rank, n);
    } catch (const std::exception& ex) {
      TORCH_CHECK(false, ex.what());
    }
    return ipc_entries_.emplace(key, std::move(e)).first->second;
  }

  Plan make_plan(int code, int rank, int64_t n) const {
    const int algo = decode_algo(code).algo;
    TORCH_CHECK(algo >= comm::kBuiltin && algo < comm::kAlgoCount, "CommEngine: unknown algorithm ", algo);
    Plan p;
    try {
      // plans are built for summation; the average is folded into the last reduce of each phase
      p = comm::build_plan(algo, topo_for(code, rank), n, 1.f / (float)topo_.world);
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
    if (force_ && topo_.world == 1) {
      // diagnostic single-rank run of the full data path: one ncclAllReduce over the 1-rank comm
      comm::Step st;
      comm::Op o;
      o.kind = comm::kColl;
      o.coll = comm::kAllReduce;
      o.comm = comm::kWorld;
      o.nsrc = 1;
      o.count = n;
      o.average = true;
      st.ops.push_back(o);
      p.steps.push_back(st);
    }
    return p;
  }

  bool staged(int algo, int dtype) const { return accum_fp32_ && dtype == kBF16 && (topo_.world > 1 || force_); }

  size_t scratch_bytes(const Plan& p, int64_t n, int dtype) const {
    return comm::staged_scratch_bytes(p.scratch_elems, n, staged(p.algo, dtype), dtype);
  }

  void ensure_scratch(size_t bytes) {
    if (scratch_.defined() && (size_t)scratch_.numel() >= bytes) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DLA_HIP_THROW(hipStreamIsCapturing(stream_->stream(), &cs));
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "CommEngine: scratch must grow during HIP-graph capture; call reserve() with the bucket sizes first");
    // Allocated with the comm stream current: the caching allocator hands a block freed here only
    // to later allocations on the same stream, i.e. in stream order after all queued work that
    // still uses the old buffer — no host synchronisation needed when replacing it.
    c10::hip::HIPStreamGuard sg(*stream_);
    size_t want = std::max(bytes, (size_t)(scratch_.defined() ? scratch_.numel() * 2 : (16 << 20)));
    scratch_ = at::empty({(int64_t)want}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device_));
  }

  // Sub-communicators exist only when both levels have more than one member (ctor): with one GPU per
  // node (L == 1) the inter-node group IS the world, with one node (K == 1) the intra-node group is.
  ncclComm_t comm_of(comm::CommId c) const {
    if (c == comm::kIntra) {
      TORCH_CHECK(intra_ || topo_.nodes() == 1, "CommEngine: intra-node communicator missing");
      return intra_ ? intra_ : comm_;
    }
    if (c == comm::kInter) {
      TORCH_CHECK(inter_ || topo_.L() == 1, "CommEngine: inter-node communicator missing");
      return inter_ ? inter_ : comm_;
    }
    return comm_;
  }

  void allreduce_on_stream(const at::Tensor& flat, int algo, bool average, const std::vector<at::Tensor>* grads,
                           const std::vector<int64_t>* offsets) {
    const int64_t n = flat.numel();
    hipStream_t st = stream_->stream();
    const int dt = flat.scalar_type() == at::kBFloat16 ? kBF16 : kF32;
    if (needs_reduce_kernel(algo))
      TORCH_CHECK(flat.scalar_type() == at::kFloat || flat.scalar_type() == at::kBFloat16,
                  "custom all-reduce algorithms support fp32/bf16 only");
    if ((topo_.world == 1 && !force_) || n == 0) {  // reference short-circuit (allreduce.py:18-19,55-56)
      if (grads) pack_tensors_on(*grads, *offsets, flat, 1.f, st);
      return;
    }
    ++n_coll_;
    if (uses_ipc(algo)) {
      allreduce_ipc(flat, algo, average, grads, offsets);
      return;
    }
    const Plan& plan = plan_for(algo, n);
    const bool stg = staged(algo, dt) && (flat.scalar_type() == at::kBFloat16);
    ensure_scratch(scratch_bytes(plan, n, dt));
    const comm::StagedLayout lay =
        comm::staged_layout(flat.data_ptr(), dt, flat.element_size(), static_cast<char*>(scratch_.data_ptr()), n, stg);
    // fp32 accumulation of a bf16 bucket: gather / cast into the fp32 staging buffer, reduce in fp32
    // on the wire and in the reduce kernels, round to bf16 once at the end.
    if (grads) {
      at::Tensor dst = stg ? at::from_blob(lay.data, {n}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_))
                           : flat;
      pack_tensors_on(*grads, *offsets, dst, 1.f, st);
    } else if (stg) {
      launch_cast(lay.data, kF32, flat.data_ptr(), kBF16, n, 1.f, st);
    }
    RcclTransport tr{*this, plan, lay, stg ? ncclFloat32 : nccl_dtype_of(flat.scalar_type()), average,
                     comm::LocalIssuer(lay.dt, lay.esz)};
    comm::execute_plan(tr, plan, st, plan_events_);
    if (stg) launch_cast(flat.data_ptr(), kBF16, lay.data, kF32, n, 1.f, st);
  }

  void allreduce_group_on_stream(const at::Tensor& group, const std::vector<int64_t>& starts,
                                 const std::vector<int64_t>& counts, int algo, bool average,
                                 const std::vector<at::Tensor>& grads, const std::vector<int64_t>& offsets) {
    hipStream_t st = stream_->stream();
    const int64_t n = group.numel();
    const int dt = group.scalar_type() == at::kBFloat16 ? kBF16 : kF32;
    if ((topo_.world == 1 && !force_) || n == 0) {
      pack_tensors_on(grads, offsets, group, 1.f, st);
      return;
    }
    const bool builtin_rccl = !uses_ipc(algo) && decode_algo(algo).algo == comm::kBuiltin;
    if (!builtin_rccl) {
      pack_tensors_on(grads, offsets, group, 1.f, st);
      for (size_t i = 0; i < starts.size(); ++i)
        if (counts[i] > 0) allreduce_on_stream(group.narrow(0, starts[i], counts[i]), algo, average, nullptr, nullptr);
      return;
    }
    if (needs_reduce_kernel(algo))
      TORCH_CHECK(group.scalar_type() == at::kFloat || group.scalar_type() == at::kBFloat16,
                  "custom all-reduce algorithms support fp32/bf16 only");
    const bool stg = staged(algo, dt) && group.scalar_type() == at::kBFloat16;
    ensure_scratch(comm::staged_scratch_bytes(0, n, stg, dt));
    char* data = stg ? static_cast<char*>(scratch_.data_ptr()) : static_cast<char*>(group.data_ptr());
    const size_t esz = stg ? 4 : (size_t)group.element_size();
    if (stg) {
      // the slot padding between members is never gathered into: zero it so the cast back writes zeros
      DLA_HIP_THROW(hipMemsetAsync(data, 0, (size_t)n * 4, st));
      at::Tensor dst = at::from_blob(data, {n}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
      pack_tensors_on(grads, offsets, dst, 1.f, st);
    } else {
      pack_tensors_on(grads, offsets, group, 1.f, st);
    }
    const ncclDataType_t ndt = stg ? ncclFloat32 : nccl_dtype_of(group.scalar_type());
    DLA_NCCL_CHECK(ncclGroupStart());
    for (size_t i = 0; i < starts.size(); ++i) {
      if (counts[i] == 0) continue;
      ++n_coll_;
      void* p = data + (size_t)starts[i] * esz;
      DLA_NCCL_CHECK(ncclAllReduce(p, p, counts[i], ndt, average ? ncclAvg : ncclSum, comm_, st));
    }
    DLA_NCCL_CHECK(ncclGroupEnd());
    if (stg) launch_cast(group.data_ptr(), kBF16, data, kF32, n, 1.f, st);
  }

  // The same Plan over peer-mapped windows (ipc.h): the bucket is staged into this rank's window
  // (fp32 for accum_fp32 bf16 buckets, else its own dtype), the plan runs there with pulls from the
  // peers' windows and flag barriers, and the result is cast / copied back into `flat`.
  void allreduce_ipc(const at::Tensor& flat, int code, bool average, const std::vector<at::Tensor>* grads,
                     const std::vector<int64_t>* offsets) {
    const int64_t n = flat.numel();
    hipStream_t st = stream_->stream();
    const int dt = flat.scalar_type() == at::kBFloat16 ? kBF16 : kF32;
    const bool stg = staged(code, dt);
    const int wdt = stg ? kF32 : dt;
    const size_t esz = wdt == kF32 ? 4 : 2;
    const IpcEntry& e = ipc_entry(code, n);
    const size_t need = comm::kIpcHeaderBytes + (size_t)e.sched.total * esz;
    TORCH_CHECK(!ipc_broken_, "CommEngine: the IPC transport was disabled after a barrier timeout");
    // The barrier tokens are host-side values baked into each barrier launch: a captured graph would
    // replay stale tokens that every peer flag already satisfies, so the barriers would pass at once.
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DLA_HIP_THROW(hipStreamIsCapturing(st, &cs));
    TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                "CommEngine: IPC all-reduces cannot be captured into a HIP graph (host-side barrier tokens); "
                "run the IPC transport eagerly (bench.py --graph off)");
    TORCH_CHECK(ipc_base_ && !ipc_peer_.empty() && need <= ipc_bytes_,
                "CommEngine: the IPC window (", ipc_bytes_, " B) does not hold this all-reduce (", need,
                " B); call reserve() with the bucket sizes first (NativeEngine.reserve maps the windows)");
    char* data = static_cast<char*>(ipc_base_) + comm::kIpcHeaderBytes;
    if (grads) {
      at::Tensor dst = at::from_blob(data, {n}, at::TensorOptions()
                                                    .dtype(wdt == kF32 ? at::kFloat : at::kBFloat16)
                                                    .device(at::kCUDA, device_));
      pack_tensors_on(*grads, *offsets, dst, 1.f, st);
    } else {
      launch_cast(data, wdt, flat.data_ptr(), dt, n, 1.f, st);
    }
    comm::LocalIssuer iss(wdt, esz);
    iss.set_stream(st);
    IpcDeviceBackend be{*this, e.sched, esz, iss};
    comm::IpcRunner<IpcDeviceBackend> run{be, e.sched, e.plans[topo_.rank], topo_.rank, average, ipc_tok_};
    IpcTransport tr{run, be, iss, e.plans[topo_.rank], average, *this};
    comm::execute_plan(tr, e.plans[topo_.rank], st, plan_events_);
    iss.set_stream(st);
    iss.flush();
    launch_cast(flat.data_ptr(), dt, data, wdt, n, 1.f, st);
  }

  struct IpcDeviceBackend {
    CommEngine& e;
    const comm::IpcSchedule& s;
    size_t esz;
    comm::LocalIssuer& iss;
    char* win(int r) const { return e.ipc_peer_[r] + comm::kIpcHeaderBytes; }
    void* ptr(int r, const comm::Ref& ref) const {
      return win(r) + (size_t)((ref.buf == comm::kData ? 0 : s.scratch_off) + ref.off) * esz;
    }
    void* tmp(int r, int64_t off) const { return win(r) + (size_t)(s.temp_off + off) * esz; }
    void barrier(uint64_t set, const std::vector<int>& wait_ranks, uint64_t wait) {
      iss.flush();
      IpcBarrier b{};
      b.mine = reinterpret_cast<uint64_t*>(e.ipc_peer_[e.topo_.rank]);
      b.set = set;
      TORCH_CHECK((int)wait_ranks.size() <= kMaxIpcPeers, "IPC barrier: too many peers");
      b.npeers = (int)wait_ranks.size();
      for (int i = 0; i < b.npeers; ++i) {
        b.peer[i] = reinterpret_cast<const uint64_t*>(e.ipc_peer_[wait_ranks[i]]);
        b.peer_rank[i] = wait_ranks[i];
      }
      b.wait = wait;
      b.err = reinterpret_cast<int*>(e.ipc_peer_[e.topo_.rank] + comm::kIpcErrOffset);
      b.diag = reinterpret_cast<uint64_t*>(e.ipc_peer_[e.topo_.rank] + comm::kIpcDiagOffset);
      b.timeout_ticks = (uint64_t)(e.timeout_s() * (double)e.wall_khz_ * 1000.0);
      launch_ipc_barrier(b, iss.stream());
    }
    void copy(void* dst, const void* src, int64_t n) { iss.copy(dst, src, n); }
    void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale) {
      iss.reduce(dst, acc, srcs, nsrc, n, scale);
    }
  };

  // plan_exec.h transport over the IPC runner: P2P steps and collectives are pulls + barriers on
  // the comm stream, local ops go through the multi-lane issuer on the given stream.
  struct IpcTransport {
    comm::IpcRunner<IpcDeviceBackend>& run;
    IpcDeviceBackend& be;
    comm::LocalIssuer& iss;
    const Plan& p;
    bool average;
    CommEngine& e;
    void coll(size_t k, hipStream_t st) {
      iss.set_stream(st);
      run.coll(k);
      iss.flush();
    }
    void transfers(size_t k, hipStream_t st) {
      iss.set_stream(st);
      run.transfers(k);
      iss.flush();
    }
    bool has_local(size_t k) const { return std::any_of(p.steps[k].ops.begin(), p.steps[k].ops.end(), comm::is_local); }
    void locals(size_t k, hipStream_t ls) {
      iss.set_stream(ls);
      const int me = e.topo_.rank;
      comm::issue_locals(p.steps[k], [&](const comm::Ref& r) { return be.ptr(me, r); }, iss, average);
      iss.flush();
    }
    hipStream_t side_stream() { return e.side_stream(); }
  };

  // The RCCL transport of plan_exec.h: collectives and P2P groups on this rank's communicators,
  // local ops through the multi-lane issuer.
  struct RcclTransport {
    CommEngine& e;
    const Plan& p;
    comm::StagedLayout lay;
    ncclDataType_t ndt;
    bool average;
    comm::LocalIssuer iss;
    void* ptr(const comm::Ref& r) const { return (r.buf == comm::kData ? lay.data : lay.scratch) + (size_t)r.off * lay.esz; }
    void coll(size_t k, hipStream_t st) {
      const comm::Op& o = p.steps[k].ops[0];
      ncclComm_t c = e.comm_of(o.comm);
      // plans are built for averaging; a summing call keeps ncclSum
      const ncclRedOp_t red = (o.average && average) ? ncclAvg : ncclSum;
      switch (o.coll) {
        case comm::kAllReduce:
          DLA_NCCL_CHECK(ncclAllReduce(ptr(o.src[0]), ptr(o.dst), o.count, ndt, red, c, st));
          break;
        case comm::kReduceScatter:
          DLA_NCCL_CHECK(ncclReduceScatter(ptr(o.src[0]), ptr(o.dst), o.count, ndt, red, c, st));
          break;
        case comm::kAllGather:
          DLA_NCCL_CHECK(ncclAllGather(ptr(o.src[0]), ptr(o.dst), o.count, ndt, c, st));
          break;
      }
    }
    void transfers(size_t k, hipStream_t st) {
      bool group = false;
      for (const auto& o : p.steps[k].ops) {
        if (o.kind != comm::kSend && o.kind != comm::kRecv) continue;
        if (!group) {
          DLA_NCCL_CHECK(ncclGroupStart());
          group = true;
        }
        if (o.kind == comm::kSend)
          DLA_NCCL_CHECK(ncclSend(ptr(o.src[0]), o.count, ndt, o.peer, e.comm_, st));
        else
          DLA_NCCL_CHECK(ncclRecv(ptr(o.dst), o.count, ndt, o.peer, e.comm_, st));
      }
      if (group) DLA_NCCL_CHECK(ncclGroupEnd());
    }
    bool has_local(size_t k) const {
      return std::any_of(p.steps[k].ops.begin(), p.steps[k].ops.end(), comm::is_local);
    }
    void locals(size_t k, hipStream_t ls) {
      iss.set_stream(ls);
      comm::issue_locals(p.steps[k], [&](const comm::Ref& r) { return ptr(r); }, iss, average);
      iss.flush();
    }
    hipStream_t side_stream() { return e.side_stream(); }
  };

  hipStream_t side_stream() {
    if (!side_)
      side_ = std::make_unique<c10::hip::HIPStream>(c10::hip::getStreamFromPool(/*isHighPriority=*/true, device_));
    return side_->stream();
  }

  int device_;
  Topology topo_;
  ncclUniqueId uid_;
  ncclComm_t comm_ = nullptr, intra_ = nullptr, inter_ = nullptr;
  bool aborted_ = false;
  bool accum_fp32_ = false;
  bool force_ = false;
  std::atomic<int64_t> n_coll_{0}, n_units_{0};  // collective_counts() (hooks issue from the autograd thread)
  std::unique_ptr<c10::hip::HIPStream> stream_;
  std::map<std::pair<int, int64_t>, Plan> plans_;
  std::map<std::pair<int, int64_t>, IpcEntry> ipc_entries_;
  void* ipc_base_ = nullptr;       // this rank's window (hipMalloc, exported)
  size_t ipc_bytes_ = 0, ipc_need_ = 0;
  std::vector<char*> ipc_peer_;    // every rank's window base as mapped here (mine = ipc_base_)
  std::vector<void*> ipc_retired_;  // superseded windows, freed once the next mapping set is verified
  uint64_t ipc_nonce_ = 0;         // identity stamp of the current window
  void* ipc_pend_base_ = nullptr;  // allocated by ipc_alloc, committed by a verified ipc_open
  size_t ipc_pend_bytes_ = 0;
  uint64_t ipc_pend_nonce_ = 0;
  int64_t ipc_generation_ = 0;     // verified mapping sets so far
  int64_t ipc_stale_ = 0;          // mappings refused because they showed the wrong nonce
  uint64_t ipc_tok_ = 0;           // barrier token counter, identical sequence on every rank
  bool ipc_broken_ = false;        // a barrier timed out: tokens are out of step, no more IPC collectives
  double timeout_s_ = 0.0;          // set_timeout
  int wall_khz_ = 100000;          // constant-clock rate for the barrier timeout
  at::Tensor scratch_;
  std::vector<hipEvent_t> ready_pool_;
  comm::EventPool plan_events_;
  std::unique_ptr<c10::hip::HIPStream> side_;
  size_t ready_next_ = 0;
  hipEvent_t last_done_ = nullptr;
  bool timing_ = false;
  std::vector<hipEvent_t> timing_events_;
  size_t used_timing_ = 0;
};

// ---------------------------------------------------------------------------------------------
// Virtual ranks: N ranks' buffers in one process, links = copies (vexec.h)
// ---------------------------------------------------------------------------------------------
// Device backend of the virtual ranks: every link copy and local op goes through the engine's
// LocalIssuer (so one step's transfers of all ranks are one multi-lane copy launch, the way one
// RCCL group carries them), and the step sequencing is the engine's own execute_plan.
struct DeviceBackend {
  std::vector<char*> data, scratch;
  size_t esz = 4;
  int dt = kF32;
  comm::LocalIssuer* iss = nullptr;
  at::TensorOptions opts;
  std::vector<at::Tensor> temps;

  void* ptr(int rank, const comm::Ref& r) {
    return (r.buf == comm::kData ? data[rank] : scratch[rank]) + (size_t)r.off * esz;
  }
  void* offset(void* p, int64_t elems) { return static_cast<char*>(p) + (size_t)elems * esz; }
  void* temp(int64_t n) {
    temps.push_back(at::empty({(int64_t)((size_t)n * esz + 256)}, opts));
    return temps.back().data_ptr();
  }
  void copy(void* dst, const void* src, int64_t n) { iss->copy(dst, src, n); }
  void zero(void* dst, int64_t n) { iss->zero(dst, n); }
  void reduce(void* dst, bool acc, const void* const* srcs, int nsrc, int64_t n, float scale) {
    iss->reduce(dst, acc, srcs, nsrc, n, scale);
  }
};

// Transport of plan_exec.h over N virtual ranks: the P2P group of a step becomes the matched copies
// of all ranks (validated by VirtualRun), collectives are emulated per communicator colour.
struct VirtualTransport {
  comm::VirtualRun<DeviceBackend>& run;
  comm::LocalIssuer& iss;
  int device;
  std::unique_ptr<c10::hip::HIPStream> side;
  void coll(size_t s, hipStream_t st) {
    iss.set_stream(st);
    run.coll(s);
    iss.flush();
  }
  void transfers(size_t s, hipStream_t st) {
    iss.set_stream(st);
    run.transfers(s);
    iss.flush();
  }
  bool has_local(size_t s) const { return run.has_local(s); }
  void locals(size_t s, hipStream_t ls) {
    iss.set_stream(ls);
    run.locals(s);
    iss.flush();
  }
  hipStream_t side_stream() {
    if (!side) side = std::make_unique<c10::hip::HIPStream>(c10::hip::getStreamFromPool(true, device));
    return side->stream();
  }
};

// All-reduce `bufs` (one tensor per virtual rank, same numel / dtype / device) in place with the
// schedules CommEngine would run for that many ranks. CUDA tensors run on the current stream
// through the engine's issuing code (execute_plan, LocalIssuer, StagedLayout); CPU tensors on the
// serial host backend. accum_fp32 stages bf16 buffers in fp32 exactly like CommEngine (cast into
// the front of each rank's scratch, fp32 plan behind it, round once). Returns the number of kernel
// launches the local ops and links took (0 on the host).
static int64_t virtual_allreduce(std::vector<at::Tensor> bufs, int algo, bool average, std::vector<std::vector<int>> rings,
                                 int local_size, std::vector<std::vector<int>> local_rings,
                                 std::vector<std::vector<int>> node_rings, bool accum_fp32) {
  const int N = (int)bufs.size();
  TORCH_CHECK(N >= 1, "virtual_allreduce: no buffers");
  const int64_t n = bufs[0].numel();
  const auto dtype = bufs[0].scalar_type();
  const bool cuda = bufs[0].is_cuda();
  for (auto& b : bufs) {
    TORCH_CHECK(b.numel() == n && b.scalar_type() == dtype && b.device() == bufs[0].device() && b.is_contiguous(),
                "virtual_allreduce: buffers must share numel, dtype, device and be contiguous");
  }
  TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16, "virtual_allreduce: fp32 / bf16 only");
  Topology t0 = make_topology(0, N, rings, local_size, local_rings, node_rings);
  cut_channels(t0, algo);
  algo = decode_algo(algo).algo;
  TORCH_CHECK(algo >= comm::kBuiltin && algo < comm::kAlgoCount, "virtual_allreduce: unknown algorithm ", algo);
  if (N == 1 || n == 0) return 0;
  std::vector<Plan> plans;
  for (int r = 0; r < N; ++r) {
    Topology t = t0;
    t.rank = r;
    try {
      plans.push_back(comm::build_plan(algo, t, n, average ? 1.f / (float)N : 1.f));
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }
  const bool stage = accum_fp32 && dtype == at::kBFloat16;
  if (cuda) {
    const int dev = bufs[0].device().index();
    c10::hip::HIPGuard guard((c10::DeviceIndex)dev);
    hipStream_t st = c10::hip::getCurrentHIPStream(dev).stream();
    const int dt = dtype == at::kBFloat16 ? kBF16 : kF32;
    DeviceBackend be;
    be.opts = at::TensorOptions().dtype(at::kByte).device(bufs[0].device());
    std::vector<at::Tensor> scr;
    std::vector<comm::StagedLayout> lay;
    for (int r = 0; r < N; ++r) {
      scr.push_back(at::empty({(int64_t)comm::staged_scratch_bytes(plans[r].scratch_elems, n, stage, dt)}, be.opts));
      lay.push_back(comm::staged_layout(bufs[r].data_ptr(), dt, bufs[r].element_size(),
                                        static_cast<char*>(scr.back().data_ptr()), n, stage));
      if (stage) launch_cast(lay[r].data, kF32, bufs[r].data_ptr(), kBF16, n, 1.f, st);
      be.data.push_back(lay[r].data);
      be.scratch.push_back(lay[r].scratch);
    }
    be.esz = lay[0].esz;
    be.dt = lay[0].dt;
    comm::LocalIssuer iss(be.dt, be.esz);
    be.iss = &iss;
    comm::VirtualRun<DeviceBackend> run(plans, t0, be);
    comm::EventPool ev;
    VirtualTransport tr{run, iss, dev, nullptr};
    try {
      run.validate();
      comm::execute_plan(tr, plans[0], st, ev);
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
    if (stage)
      for (int r = 0; r < N; ++r) launch_cast(bufs[r].data_ptr(), kBF16, lay[r].data, kF32, n, 1.f, st);
    // temporaries of the emulated collectives are freed with `be`: their last use is queued on `st`
    // (the side stream only runs plan-local ops on rank buffers), which the caching allocator orders
    return iss.launches();
  }
  comm::HostBackend be;
  std::vector<std::vector<char>> stage_mem, scr;
  be.bf16 = dtype == at::kBFloat16 && !stage;
  be.esz = be.bf16 ? 2 : 4;
  for (int r = 0; r < N; ++r) {
    if (stage) {
      stage_mem.emplace_back((size_t)n * 4);
      float* f = reinterpret_cast<float*>(stage_mem.back().data());
      const uint16_t* b = static_cast<const uint16_t*>(bufs[r].data_ptr());
      for (int64_t i = 0; i < n; ++i) f[i] = comm::HostBackend::b2f(b[i]);
      be.data.push_back(stage_mem.back().data());
    } else {
      be.data.push_back(static_cast<char*>(bufs[r].data_ptr()));
    }
    scr.emplace_back((size_t)plans[r].scratch_elems * be.esz + 64);
    be.scratch.push_back(scr.back().data());
  }
  comm::VirtualRun<comm::HostBackend> run(plans, t0, be);
  try {
    run.run();
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  if (stage) {
    for (int r = 0; r < N; ++r) {
      const float* f = reinterpret_cast<const float*>(stage_mem[r].data());
      uint16_t* b = static_cast<uint16_t*>(bufs[r].data_ptr());
      for (int64_t i = 0; i < n; ++i) b[i] = comm::HostBackend::f2b(f[i]);
    }
  }
  return 0;
}

// All-reduce host buffers (one CPU tensor per rank) through the IPC protocol of ipc.h with one
// thread per rank and atomic flags: the schedule matching and barrier protocol the GPU transport
// runs, checked under real concurrency in the CPU test suite.
static void ipc_host_allreduce(std::vector<at::Tensor> bufs, int code, bool average, std::vector<std::vector<int>> rings,
                               int local_size, std::vector<std::vector<int>> local_rings,
                               std::vector<std::vector<int>> node_rings, bool accum_fp32, double timeout_s) {
  const int N = (int)bufs.size();
  TORCH_CHECK(N >= 1, "ipc_host_allreduce: no buffers");
  const int64_t n = bufs[0].numel();
  const auto dtype = bufs[0].scalar_type();
  for (auto& b : bufs)
    TORCH_CHECK(!b.is_cuda() && b.numel() == n && b.scalar_type() == dtype && b.is_contiguous(),
                "ipc_host_allreduce: contiguous CPU buffers of one numel / dtype");
  TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16, "ipc_host_allreduce: fp32 / bf16 only");
  if (N == 1 || n == 0) return;
  Topology t0 = make_topology(0, N, rings, local_size, local_rings, node_rings);
  cut_channels(t0, code);
  const int algo = decode_algo(code).algo;
  std::vector<Plan> plans;
  for (int r = 0; r < N; ++r) {
    Topology t = t0;
    t.rank = r;
    try {
      plans.push_back(comm::build_plan(algo, t, n, 1.f / (float)N));
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }
  std::vector<comm::IpcSchedule> sch;
  for (int r = 0; r < N; ++r) {
    Topology t = t0;
    t.rank = r;
    try {
      sch.push_back(comm::build_ipc_schedule(plans, t, r, n));
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }
  const bool stage = accum_fp32 && dtype == at::kBFloat16;
  comm::IpcHostShared sh(N);
  sh.bf16 = dtype == at::kBFloat16 && !stage;
  sh.esz = sh.bf16 ? 2 : 4;
  sh.scratch_off = sch[0].scratch_off;
  sh.temp_off = sch[0].temp_off;
  sh.timeout_s = timeout_s;
  for (int r = 0; r < N; ++r) {
    sh.windows[r].assign((size_t)sch[r].total * sh.esz + 64, 0);
    char* w = sh.windows[r].data();
    if (stage) {
      const uint16_t* b = static_cast<const uint16_t*>(bufs[r].data_ptr());
      for (int64_t i = 0; i < n; ++i) reinterpret_cast<float*>(w)[i] = comm::HostBackend::b2f(b[i]);
    } else {
      std::memcpy(w, bufs[r].data_ptr(), (size_t)n * sh.esz);
    }
  }
  std::vector<std::string> errs(N);
  {
    pybind11::gil_scoped_release nogil;
    std::vector<std::thread> th;
    for (int r = 0; r < N; ++r)
      th.emplace_back([&, r] {
        try {
          comm::IpcHostBackend be{sh, r};
          uint64_t tok = 0;
          comm::ipc_host_run(be, sch[r], plans[r], average, tok);
        } catch (const std::exception& e) {
          errs[r] = e.what();
          sh.timeout_s = 0.0;  // let the other ranks fail fast instead of waiting out the timeout
        }
      });
    for (auto& x : th) x.join();
  }
  for (int r = 0; r < N; ++r) TORCH_CHECK(errs[r].empty(), "ipc_host_allreduce rank ", r, ": ", errs[r]);
  for (int r = 0; r < N; ++r) {
    const char* w = sh.windows[r].data();
    if (stage) {
      uint16_t* b = static_cast<uint16_t*>(bufs[r].data_ptr());
      for (int64_t i = 0; i < n; ++i) b[i] = comm::HostBackend::f2b(reinterpret_cast<const float*>(w)[i]);
    } else {
      std::memcpy(bufs[r].data_ptr(), w, (size_t)n * sh.esz);
    }
  }
}

static std::string plan_describe(int algo, int rank, int world, int64_t n, std::vector<std::vector<int>> rings,
                                 int local_size, std::vector<std::vector<int>> local_rings,
                                 std::vector<std::vector<int>> node_rings, bool average) {
  Topology t = make_topology(rank, world, std::move(rings), local_size, std::move(local_rings), std::move(node_rings));
  cut_channels(t, algo);
  algo = decode_algo(algo).algo;
  try {
    return comm::describe(comm::build_plan(algo, t, n, average ? 1.f / (float)world : 1.f));
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  return "";
}

void bind_comm(pybind11::module& m) {
  using VV = std::vector<std::vector<int>>;
  pybind11::class_<CommEngine>(m, "CommEngine")
      .def(pybind11::init<int, int, pybind11::bytes, int, VV, int, VV, VV>(), pybind11::arg("rank"),
           pybind11::arg("world"), pybind11::arg("unique_id"), pybind11::arg("device"), pybind11::arg("rings"),
           pybind11::arg("local_size") = 0, pybind11::arg("local_rings") = VV{}, pybind11::arg("node_rings") = VV{})
      .def_static("get_unique_id", &CommEngine::get_unique_id)
      .def("rank", &CommEngine::rank)
      .def("world", &CommEngine::world)
      .def("local_size", &CommEngine::local_size)
      .def("num_rings", &CommEngine::num_rings)
      .def("set_accum_fp32", &CommEngine::set_accum_fp32)
      .def("set_force", &CommEngine::set_force)
      .def("accum_fp32", &CommEngine::accum_fp32)
      .def("join_current", &CommEngine::join_current)
      .def("wait_on_current", &CommEngine::wait_on_current)
      .def("synchronize", &CommEngine::synchronize)
      .def("async_error", &CommEngine::async_error)
      .def("abort", &CommEngine::abort)
      .def("aborted", &CommEngine::aborted)
      .def("stream_handle", &CommEngine::stream_handle)
      .def("reserve", &CommEngine::reserve, pybind11::arg("algo"), pybind11::arg("sizes"), pybind11::arg("dtype"))
      .def("describe_plan", &CommEngine::describe_plan)
      .def("allreduce", &CommEngine::allreduce, pybind11::arg("flat"), pybind11::arg("algo"), pybind11::arg("average"))
      .def("bucket_allreduce", &CommEngine::bucket_allreduce, pybind11::arg("flat"), pybind11::arg("algo"),
           pybind11::arg("average"), pybind11::arg("table").none(true), pybind11::arg("pack_scale") = 1.0,
           pybind11::arg("unpack_scale") = 1.0)
      .def("bucket_allreduce_list", &CommEngine::bucket_allreduce_list, pybind11::arg("flat"), pybind11::arg("algo"),
           pybind11::arg("average"), pybind11::arg("grads"), pybind11::arg("offsets"))
      .def("bucket_allreduce_group", &CommEngine::bucket_allreduce_group, pybind11::arg("group"),
           pybind11::arg("starts"), pybind11::arg("counts"), pybind11::arg("algo"), pybind11::arg("average"),
           pybind11::arg("grads"), pybind11::arg("offsets"))
      .def("broadcast", &CommEngine::broadcast)
      .def("allgather", &CommEngine::allgather)
      .def("set_timing", &CommEngine::set_timing)
      .def("consume_comm_ms", &CommEngine::consume_comm_ms)
      .def("collective_counts", &CommEngine::collective_counts, pybind11::arg("reset") = false)
      .def("has_rccl", &CommEngine::has_rccl)
      .def("rccl_count", &CommEngine::rccl_count)
      .def("ipc_need", &CommEngine::ipc_need)
      .def("ipc_capacity", &CommEngine::ipc_capacity)
      .def("ipc_alloc", &CommEngine::ipc_alloc)
      .def("ipc_open", &CommEngine::ipc_open)
      .def("ipc_error", &CommEngine::ipc_error)
      .def("ipc_error_info", &CommEngine::ipc_error_info)
      .def("set_timeout", &CommEngine::set_timeout)
      .def("timeout_s", &CommEngine::timeout_s);
  m.def("ipc_host_allreduce", &ipc_host_allreduce,
        "all-reduce CPU buffers with the IPC transport's pull/barrier protocol, one thread per rank",
        pybind11::arg("bufs"), pybind11::arg("algo"), pybind11::arg("average") = true, pybind11::arg("rings") = VV{},
        pybind11::arg("local_size") = 0, pybind11::arg("local_rings") = VV{}, pybind11::arg("node_rings") = VV{},
        pybind11::arg("accum_fp32") = false, pybind11::arg("timeout_s") = 30.0);
  m.attr("ALGO_IPC_FLAG") = 256;
  m.attr("ALGO_CHANNEL_SHIFT") = 4;
  m.def("virtual_allreduce", &virtual_allreduce, "all-reduce N virtual ranks' buffers with the engine's schedules",
        pybind11::arg("bufs"), pybind11::arg("algo"), pybind11::arg("average") = true, pybind11::arg("rings") = VV{},
        pybind11::arg("local_size") = 0, pybind11::arg("local_rings") = VV{}, pybind11::arg("node_rings") = VV{},
        pybind11::arg("accum_fp32") = false);
  m.def("plan_describe", &plan_describe, pybind11::arg("algo"), pybind11::arg("rank"), pybind11::arg("world"),
        pybind11::arg("n"), pybind11::arg("rings") = VV{}, pybind11::arg("local_size") = 0,
        pybind11::arg("local_rings") = VV{}, pybind11::arg("node_rings") = VV{}, pybind11::arg("average") = true);
  m.attr("ALGO_BUILTIN") = (int)comm::kBuiltin;
  m.attr("ALGO_RING") = (int)comm::kRing;
  m.attr("ALGO_DIRECT") = (int)comm::kDirect;
  m.attr("ALGO_CENTRAL") = (int)comm::kCentral;
  m.attr("ALGO_RSAG") = (int)comm::kRsAg;
  m.attr("ALGO_HIER_RING") = (int)comm::kHierRing;
  m.attr("ALGO_HIER_COLL") = (int)comm::kHierColl;
  m.attr("ALGO_RING_PIPE") = (int)comm::kRingPipe;
  m.attr("ALGO_HIER_CENTRAL") = (int)comm::kHierCentral;
}

}  // namespace dla
