// Host-side checks of the comm engine's pure C++ parts, built as a standalone executable so it can run under
// AddressSanitizer + UndefinedBehaviorSanitizer on the CPU (the GPU pool runs no sanitizers):
//   * plan.cpp       -- every schedule (build_plan) at N = 2..8, every local size the 2-step algorithms take,
//                       1..3 ring channels, odd and tiny bucket sizes, average on / off;
//   * vexec.h        -- the lockstep virtual-rank executor over HostBackend (fp32 and bf16 storage), checked
//                       exactly against an fp64 oracle of the all-reduce;
//   * ipc.h          -- the IPC pull / flag-barrier protocol with one thread per rank over IpcHostBackend
//                       (real concurrency, atomics), the same oracle; plus a rank that never arrives, which must
//                       surface as a barrier-timeout exception on the others (no hang, no stray access).
// The Python tests (tests/test_comm_plans.py, test_ipc_protocol.py) drive the same code through _C.so; this
// binary exercises it without Python so the sanitizer runtime owns the process.
//
// Build + run: python -m distributed_learning_amd._build --sanitize   (g++ -fsanitize=address,undefined)
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../comm/ipc.h"
#include "../comm/plan.h"
#include "../comm/vexec.h"

using namespace dla::comm;

namespace {

int g_cases = 0, g_fail = 0;

void check(bool ok, const std::string& what) {
  ++g_cases;
  if (!ok) {
    ++g_fail;
    std::fprintf(stderr, "FAIL %s\n", what.c_str());
  }
}

// channel ring orders over n ranks: order c visits i * s_c + c (mod n) for steps s_c coprime with n
std::vector<std::vector<int>> rings_for(int n, int channels) {
  std::vector<std::vector<int>> out;
  for (int s = 1; (int)out.size() < channels && s < 4 * n; ++s) {
    int a = s, b = n;
    while (b) {
      const int t = a % b;
      a = b;
      b = t;
    }
    if (a != 1) continue;
    std::vector<int> o(n);
    for (int i = 0; i < n; ++i) o[i] = (int)(((int64_t)i * s + (int64_t)out.size()) % n);
    out.push_back(o);
  }
  if (out.empty()) {
    std::vector<int> o(n);
    for (int i = 0; i < n; ++i) o[i] = i;
    out.push_back(o);
  }
  return out;
}

Topology topo(int N, int L, int channels, int rank) {
  Topology t;
  t.world = N;
  t.rank = rank;
  t.local_size = L;
  t.rings = rings_for(N, channels);
  t.local_rings = rings_for(L, std::min(channels, std::max(1, L - 1)));
  t.node_rings = rings_for(N / L, std::min(channels, std::max(1, N / L - 1)));
  return t;
}

// exactly representable inputs: (i % 7 - 3) * (rank + 1); the sum over ranks is (i % 7 - 3) N (N + 1) / 2
float input(int64_t i, int r) { return (float)(((i % 7) - 3) * (r + 1)); }
double expect(int64_t i, int N, bool average) {
  const double s = (double)((i % 7) - 3) * N * (N + 1) / 2.0;
  return average ? s / N : s;
}

std::vector<Plan> plans_for(int algo, int N, int L, int ch, int64_t n, bool average) {
  std::vector<Plan> plans;
  for (int r = 0; r < N; ++r) plans.push_back(build_plan(algo, topo(N, L, ch, r), n, average ? 1.f / (float)N : 1.f));
  return plans;
}

void run_vexec(int algo, int N, int L, int ch, int64_t n, bool bf16, bool average) {
  const std::string tag = std::string("vexec ") + algo_name(algo) + " N=" + std::to_string(N) + " L=" +
                          std::to_string(L) + " ch=" + std::to_string(ch) + " n=" + std::to_string(n) +
                          (bf16 ? " bf16" : " fp32") + (average ? " avg" : " sum");
  std::vector<Plan> plans;
  try {
    plans = plans_for(algo, N, L, ch, n, average);
  } catch (const std::exception& e) {
    check(false, tag + ": build_plan threw " + e.what());
    return;
  }
  HostBackend be;
  be.bf16 = bf16;
  be.esz = bf16 ? 2 : 4;
  std::vector<std::vector<char>> data(N), scr(N);
  for (int r = 0; r < N; ++r) {
    data[r].assign((size_t)n * be.esz, 0);
    for (int64_t i = 0; i < n; ++i) be.store(data[r].data(), i, input(i, r));
    scr[r].assign((size_t)plans[r].scratch_elems * be.esz + 64, 0);
    be.data.push_back(data[r].data());
    be.scratch.push_back(scr[r].data());
  }
  try {
    VirtualRun<HostBackend> run(plans, topo(N, L, ch, 0), be);
    run.run();
  } catch (const std::exception& e) {
    check(false, tag + ": run threw " + e.what());
    return;
  }
  double worst = 0;
  for (int r = 0; r < N; ++r)
    for (int64_t i = 0; i < n; ++i) worst = std::max(worst, std::fabs(be.load(data[r].data(), i) - expect(i, N, average)));
  // fp32: exact integers, averages within 1 ulp-ish; bf16: 8 significant bits of values up to 3 N (N+1) / 2
  const double tol = bf16 ? 0.02 * 3.0 * N * (N + 1) / 2.0 : 1e-5 * N * N;
  check(worst <= tol, tag + ": worst error " + std::to_string(worst));
  (void)describe(plans[0]);
}

void run_ipc(int algo, int N, int L, int ch, int64_t n, bool average, bool drop_rank) {
  const std::string tag = std::string("ipc ") + algo_name(algo) + " N=" + std::to_string(N) + " L=" +
                          std::to_string(L) + " ch=" + std::to_string(ch) + " n=" + std::to_string(n) +
                          (drop_rank ? " (rank N-1 never arrives)" : "");
  std::vector<Plan> plans;
  std::vector<IpcSchedule> sch;
  try {
    plans = plans_for(algo, N, L, ch, n, true);
    for (int r = 0; r < N; ++r) sch.push_back(build_ipc_schedule(plans, topo(N, L, ch, r), r, n));
  } catch (const std::exception& e) {
    check(false, tag + ": schedule threw " + e.what());
    return;
  }
  IpcHostShared sh(N);
  sh.esz = 4;
  sh.scratch_off = sch[0].scratch_off;
  sh.temp_off = sch[0].temp_off;
  sh.timeout_s = drop_rank ? 0.5 : 30.0;
  for (int r = 0; r < N; ++r) {
    sh.windows[r].assign((size_t)sch[r].total * sh.esz + 64, 0);
    float* w = reinterpret_cast<float*>(sh.windows[r].data());
    for (int64_t i = 0; i < n; ++i) w[i] = input(i, r);
  }
  std::vector<std::string> errs(N);
  std::vector<std::thread> th;
  for (int r = 0; r < N; ++r) {
    if (drop_rank && r == N - 1) continue;
    th.emplace_back([&, r] {
      try {
        IpcHostBackend be{sh, r};
        uint64_t tok = 0;
        ipc_host_run(be, sch[r], plans[r], average, tok);
      } catch (const std::exception& e) {
        errs[r] = e.what();
      }
    });
  }
  for (auto& x : th) x.join();
  if (drop_rank) {
    bool any = false;
    for (int r = 0; r < N - 1; ++r) any = any || errs[r].find("never arrived") != std::string::npos;
    check(any, tag + ": no rank reported the missing peer");
    return;
  }
  for (int r = 0; r < N; ++r) check(errs[r].empty(), tag + " rank " + std::to_string(r) + ": " + errs[r]);
  double worst = 0;
  for (int r = 0; r < N; ++r) {
    const float* w = reinterpret_cast<const float*>(sh.windows[r].data());
    for (int64_t i = 0; i < n; ++i) worst = std::max(worst, std::fabs(w[i] - expect(i, N, average)));
  }
  check(worst <= 1e-5 * N * N, tag + ": worst error " + std::to_string(worst));
}

void bad_inputs() {
  // a topology whose ring is not a permutation, and plans of two different algorithms, must throw
  Topology t = topo(4, 4, 1, 0);
  t.rings = {{0, 1, 1, 3}};
  bool threw = false;
  try {
    (void)build_plan(kRing, t, 100, 0.25f);
  } catch (const std::exception&) {
    threw = true;
  }
  check(threw, "invalid ring order accepted");
  std::vector<Plan> plans;
  for (int r = 0; r < 4; ++r) plans.push_back(build_plan(r == 2 ? kDirect : kRing, topo(4, 4, 1, r), 1000, 0.25f));
  HostBackend be;
  std::vector<std::vector<char>> data(4), scr(4);
  for (int r = 0; r < 4; ++r) {
    data[r].assign(4000, 0);
    scr[r].assign((size_t)plans[r].scratch_elems * 4 + 64, 0);
    be.data.push_back(data[r].data());
    be.scratch.push_back(scr[r].data());
  }
  threw = false;
  try {
    VirtualRun<HostBackend> run(plans, topo(4, 4, 1, 0), be);
    run.run();
  } catch (const std::exception&) {
    threw = true;
  }
  check(threw, "mismatched plans executed without an error");
}

}  // namespace

int main() {
  const int64_t sizes[] = {1, 5, 257, 4099};
  for (int N : {2, 3, 4, 5, 6, 8}) {
    for (int algo = 0; algo < kAlgoCount; ++algo) {
      const bool hier = algo == kHierRing || algo == kHierColl || algo == kHierCentral;
      std::vector<int> locals{N};
      if (hier)
        for (int L = 1; L < N; ++L)
          if (N % L == 0) locals.push_back(L);
      for (int L : locals)
        for (int ch = 1; ch <= std::min(3, std::max(1, N - 1)); ++ch)
          for (int64_t n : sizes) {
            run_vexec(algo, N, L, ch, n, false, true);
            run_vexec(algo, N, L, ch, n, false, false);
            run_vexec(algo, N, L, ch, n, true, true);
            if (n >= 257) run_ipc(algo, N, L, ch, n, true, false);
          }
    }
  }
  run_ipc(kRing, 4, 4, 1, 1000, true, true);
  run_ipc(kDirect, 3, 3, 1, 1000, true, true);
  bad_inputs();
  std::printf("host_check: %d cases, %d failed\n", g_cases, g_fail);
  return g_fail ? 1 : 0;
}
