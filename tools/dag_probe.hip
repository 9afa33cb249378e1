// Probe of the persistent dataflow Cholesky (diagnostic; includes the shipped gpx_potrf.hip + gpx_potrf_dag.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        dag_probe.hip -o dag_probe
// Usage: dag_probe [n] [reps] [batch]
// Prints: factor agreement with the multi-launch schedule, ||L L^T - A|| on sampled rows, D_k L_kk - I, batched vs single
// bit-equality, NOT_PD and timeout reporting, hipEvent times of both schedules, and the chain's per-step timeline.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <vector>
#include <algorithm>
#include <cmath>
#include <climits>
#include "gpx_internal.h"
__device__ unsigned long long g_chain[64][10];
__device__ unsigned long long g_task[16384][5];
__device__ int g_task_wg[16384];
#define GPX_DAG_STAMP(kind, a, b, s) do { if (threadIdx.x == 0 && blockIdx.y == 0) g_chain[a][s] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define GPX_DAG_TASK_STAMP(idx, s) do { if (threadIdx.x == 0 && blockIdx.y == 0 && idx < 16384) { g_task[idx][s] = __builtin_amdgcn_s_memrealtime(); g_task_wg[idx] = blockIdx.x; } } while (0)
namespace gpx {
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
#include "gpx_potrf_dag.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void make_gram(int n, int seed, std::vector<double>& K, double noise) {
  const int d = 8;
  std::vector<double> X((size_t)n * d);
  unsigned long long s = 88172645463325252ull + seed * 7919ull;
  for (auto& x : X) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (double)(s >> 11) / 9007199254740992.0; }
  const double ls = exp(sqrt(2.0) + 0.5 * log((double)d) - 3.0);
  K.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double r2 = 0;
      for (int k = 0; k < d; ++k) { const double t = (X[i * d + k] - X[j * d + k]) / ls; r2 += t * t; }
      const double v = exp(-0.5 * r2) + (i == j ? noise : 0.0);
      K[(size_t)i * n + j] = v;
      K[(size_t)j * n + i] = v;
    }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int batch = argc > 3 ? atoi(argv[3]) : 4;
  const int nblk = n / NB;
  std::vector<double> K;
  make_gram(n, 1, K, 1e-4);
  const size_t bytes = (size_t)n * n * 8, dbytes = (size_t)2 * nblk * NB * NB * 8;
  double *A, *Aref, *D, *Dref;
  int32_t* info;
  CK(hipMalloc(&A, bytes * batch));
  CK(hipMalloc(&Aref, bytes));
  CK(hipMalloc(&D, dbytes * batch));
  CK(hipMalloc(&Dref, dbytes));
  CK(hipMalloc(&info, 4 * batch));
  Context ctx;
  CK(hipStreamCreate(&ctx.stream));
  Batch one;
  auto run = [&](int sched, double* a, double* d, const Batch& bt) {
    ctx.potrf_schedule = sched;
    CK(hipMemsetAsync(info, 0, 4 * bt.count, ctx.stream));
    CK(launch_potrf(&ctx, n, a, n, d, info, bt, nullptr, 0));
  };
  // reference: multi-launch
  CK(hipMemcpy(Aref, K.data(), bytes, hipMemcpyHostToDevice));
  run(1, Aref, Dref, one);
  CK(hipStreamSynchronize(ctx.stream));
  int hinfo = 0;
  CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
  printf("n=%d multi-launch info=%d\n", n, hinfo);
  // dataflow
  CK(hipMemcpy(A, K.data(), bytes, hipMemcpyHostToDevice));
  printf("dag workers per problem: %d (cus %d)\n", potrf_dag_workers(&ctx, n, 1), ctx.cu_count);
  run(2, A, D, one);
  CK(hipStreamSynchronize(ctx.stream));
  CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
  printf("dag info=%d\n", hinfo);
  std::vector<double> L((size_t)n * n), Lr((size_t)n * n), Dh(nblk * NB * NB), Dr(nblk * NB * NB);
  CK(hipMemcpy(L.data(), A, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(Lr.data(), Aref, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(Dh.data(), D, Dh.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(Dr.data(), Dref, Dr.size() * 8, hipMemcpyDeviceToHost));
  double dmax = 0, lmax = 0, ddmax = 0;
  long nbad = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      const double a = L[(size_t)i * n + j], b = Lr[(size_t)i * n + j];
      if (!std::isfinite(a)) ++nbad;
      dmax = std::max(dmax, fabs(a - b));
      lmax = std::max(lmax, fabs(b));
    }
  for (size_t e = 0; e < Dh.size(); ++e) ddmax = std::max(ddmax, fabs(Dh[e] - Dr[e]));
  printf("max|L_dag - L_multi| = %.3e (max|L| %.3e), non-finite %ld, max|D_dag - D_multi| = %.3e\n", dmax, lmax, nbad,
         ddmax);
  // residual on sampled rows: (L L^T)[i][j] - K[i][j]
  double res = 0;
  for (int i = 0; i < n; i += std::max(1, n / 97))
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += L[(size_t)i * n + k] * L[(size_t)j * n + k];
      res = std::max(res, fabs(s - K[(size_t)i * n + j]));
    }
  printf("max|L L^T - K| (sampled rows) = %.3e\n", res);
  // D_k L_kk - I
  double dres = 0;
  for (int k = 0; k < nblk; ++k)
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        double s = 0;
        for (int m = 0; m < NB; ++m) s += Dh[(size_t)k * NB * NB + i * NB + m] * L[(size_t)(k * NB + m) * n + k * NB + j];
        dres = std::max(dres, fabs(s - (i == j)));
      }
  printf("max|D_k L_kk - I| = %.3e\n", dres);
  // timeline of the single run
  {
    unsigned long long ch[64][10];
    CK(hipMemcpyFromSymbol(ch, HIP_SYMBOL(g_chain), sizeof(ch)));
    const unsigned long long t0 = ch[0][0];
    // phases: 0 start, 1 S row (wave 0), 2 U00 + S rows of all waves, 3..6 pivot-block barriers, 7 end of factor,
    // 8 out published, 9 next tiles ready (next step's 0)
    const char* names[9] = {"S", "U00", "chol0", "blk1", "blk2", "blk3", "tail", "out", "next"};
    double acc[9] = {0};
    int nst = 0;
    for (int c = 1; c + 1 < nblk; ++c) {
      for (int p = 0; p < 9; ++p) acc[p] += ((double)ch[c][p + 1] - (double)ch[c][p]) * 0.01;
      ++nst;
    }
    printf("chain: total %.1f us, %.2f us per step; phase averages:", (ch[nblk - 1][8] - t0) * 0.01,
           (ch[nblk - 1][0] - ch[1][0]) * 0.01 / (nblk - 2));
    for (int p = 0; p < 9; ++p) printf(" %s %.2f", names[p], acc[p] / nst);
    printf("\n");
    for (int c = 1; c < nblk; c += std::max(1, nblk / 16)) {
      printf("  c=%2d start %8.2f:", c, (ch[c][0] - t0) * 0.01);
      for (int p = 0; p < 9 && (p < 8 || c + 1 < nblk); ++p) printf(" %s %5.2f", names[p], ((double)ch[c][p + 1] - (double)ch[c][p]) * 0.01);
      printf("\n");
    }
    auto* cache = reinterpret_cast<dag::Cache*>(ctx.dag_cache);
    const dag::Plan& plan = *cache->plans.begin()->second;
    const int nt = (int)plan.list.size();
    static unsigned long long tk[16384][5];
    CK(hipMemcpyFromSymbol(tk, HIP_SYMBOL(g_task), sizeof(tk)));
    double busy[4] = {0}, run[4] = {0}, cnt[4] = {0}, tend = 0, frw2 = 0;
    for (int q = 0; q < nt && q < 16384; ++q) {
      const int type = plan.list[q] & 0xff;
      busy[type] += (tk[q][1] - tk[q][0]) * 0.01;
      run[type] += (tk[q][1] - tk[q][2]) * 0.01;
      if (type == 1) { run[type] -= (tk[q][4] - tk[q][3]) * 0.01; frw2 += (tk[q][4] - tk[q][3]) * 0.01; }
      cnt[type] += 1;
      tend = std::max(tend, (tk[q][1] - t0) * 0.01);
    }
    printf("tasks %d (sim %.1f us): FR %.0f avg %.2f us (running %.2f, waiting for L_{k+1,k} %.2f), U64 %.0f avg %.2f (running %.2f), U128 %.0f avg %.2f (running %.2f); last task end %.1f us\n",
           nt, plan.sim_us, cnt[1], busy[1] / std::max(1.0, cnt[1]), run[1] / std::max(1.0, cnt[1]), frw2 / std::max(1.0, cnt[1]),
           cnt[2], busy[2] / std::max(1.0, cnt[2]), run[2] / std::max(1.0, cnt[2]), cnt[3],
           busy[3] / std::max(1.0, cnt[3]), run[3] / std::max(1.0, cnt[3]), tend);
    double kb[9] = {0}, kc[9] = {0};
    for (int q = 0; q < nt && q < 16384; ++q)
      if ((plan.list[q] & 0xff) == 3) {
        const int K = (int)((plan.list[q] >> 32) & 0xff) - (int)((plan.list[q] >> 24) & 0xff);
        kb[K] += (tk[q][1] - tk[q][2]) * 0.01;
        kc[K] += 1;
      }
    // the critical hand-off: chain step c publishes L_{c,c-1} (after pivot block 0), FR(c+1, c-1) (critical list entry
    // c-1) updates A_{c+1,c} and A_{c+1,c+1}, the chain loads them after its step; times relative to step c's start
    printf("critical FR(c+1,c-1) vs chain step c (us from step start): L_{c,c-1} pub | FR taken, deps met, L_ik pub, "
           "end | chain out, next ready\n");
    for (int c = 2; c + 1 < nblk; c += std::max(1, nblk / 12)) {
      const int q = c - 1;
      if (q >= plan.lend[0]) break;
      const double b0 = (double)ch[c][0];
      auto rel = [&](unsigned long long x) { return ((double)x - b0) * 0.01; };
      printf("  c=%2d: %6.2f | %7.2f %7.2f %7.2f %7.2f | %6.2f %6.2f\n", c, rel(ch[c][3]), rel(tk[q][0]), rel(tk[q][2]),
             rel(tk[q][3]), rel(tk[q][1]), rel(ch[c][8]), rel(ch[c][9]));
    }
    for (int K = 1; K <= 8; ++K) if (kc[K] > 0) printf("  U128 K=%d: %4.0f tasks, running avg %.2f us\n", K, kc[K], kb[K] / kc[K]);
  }
  // timing
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int sched = 1; sched <= 2; ++sched) {
    float best = 1e9, tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpy(A, K.data(), bytes, hipMemcpyHostToDevice));
      CK(hipEventRecord(e0, ctx.stream));
      run(sched, A, D, one);
      CK(hipEventRecord(e1, ctx.stream));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      tot += ms;
    }
    printf("schedule %s: potrf best %.3f ms, mean %.3f ms\n", sched == 1 ? "multi-launch" : "dataflow", best, tot / reps);
  }
  // batched bit-equality
  if (batch > 1) {
    for (int b = 0; b < batch; ++b) {
      std::vector<double> Kb;
      make_gram(n, 1 + b, Kb, 1e-4);
      CK(hipMemcpy(A + (size_t)b * n * n, Kb.data(), bytes, hipMemcpyHostToDevice));
    }
    Batch bt;
    bt.count = batch;
    bt.k = (int64_t)n * n;
    bt.dinv = 2 * nblk * NB * NB;
    printf("batched workers per problem: %d\n", potrf_dag_workers(&ctx, n, batch));
    // the first call builds the plan (host simulation); time the later ones, each on fresh copies of the Grams
    float ms = 1e9;
    double* Ab = nullptr;
    CK(hipMalloc(&Ab, bytes * batch));
    CK(hipMemcpy(Ab, A, bytes * batch, hipMemcpyDeviceToDevice));
    auto t0 = std::chrono::steady_clock::now();
    run(2, A, D, bt);
    CK(hipStreamSynchronize(ctx.stream));
    printf("batched first call (plan build + factor): %.3f ms\n",
           std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    for (int r = 0; r < std::max(1, reps); ++r) {
      CK(hipMemcpy(A, Ab, bytes * batch, hipMemcpyDeviceToDevice));
      float m;
      CK(hipEventRecord(e0, ctx.stream));
      run(2, A, D, bt);
      CK(hipEventRecord(e1, ctx.stream));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&m, e0, e1));
      ms = std::min(ms, m);
    }
    CK(hipFree(Ab));
    std::vector<int32_t> hi(batch);
    CK(hipMemcpy(hi.data(), info, 4 * batch, hipMemcpyDeviceToHost));
    int mism = 0;
    for (int b = 0; b < batch; ++b) {
      std::vector<double> Kb, Lb((size_t)n * n), Ls((size_t)n * n);
      make_gram(n, 1 + b, Kb, 1e-4);
      CK(hipMemcpy(Lb.data(), A + (size_t)b * n * n, bytes, hipMemcpyDeviceToHost));
      CK(hipMemcpy(Aref, Kb.data(), bytes, hipMemcpyHostToDevice));
      run(2, Aref, Dref, one);
      CK(hipStreamSynchronize(ctx.stream));
      CK(hipMemcpy(Ls.data(), Aref, bytes, hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) mism += memcmp(&Lb[(size_t)i * n + j], &Ls[(size_t)i * n + j], 8) != 0;
    }
    printf("batched x%d: best %.3f ms, info %d %d.., lower entries differing from single fits: %d\n", batch, ms, hi[0],
           batch > 1 ? hi[1] : 0, mism);
  }
  // forward substitution folded into the factorisation: z = L^{-1} (Y - mean) against a host substitution with the
  // device's own L (1 and 3 right-hand sides, n - 5 real rows so that the padding is exercised)
  for (int nrhs : {1, 3}) {
    const int nr = nrhs == 1 ? 1 : GPX_MAX_RHS;
    const int nreal = n - 5;
    const double mean = 0.25;
    std::vector<double> Yh((size_t)nreal * nrhs);
    for (size_t e = 0; e < Yh.size(); ++e) Yh[e] = std::sin(0.37 * (double)e) + 0.1 * (double)(e % 7);
    double *Yd = nullptr, *fb = nullptr;
    CK(hipMalloc(&Yd, Yh.size() * 8));
    CK(hipMalloc(&fb, (size_t)2 * n * nr * 8));
    CK(hipMemcpy(Yd, Yh.data(), Yh.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(A, K.data(), bytes, hipMemcpyHostToDevice));
    ForwardRhs fr;
    fr.Y = Yd;
    fr.ldy = nrhs;
    fr.nrhs = nrhs;
    fr.n = nreal;
    fr.mean = mean;
    fr.buf = fb;
    bool zd = false;
    ctx.potrf_schedule = 2;
    CK(hipMemsetAsync(info, 0, 4, ctx.stream));
    CK(launch_potrf(&ctx, n, A, n, D, info, one, nullptr, 0, &fr, &zd));
    CK(hipStreamSynchronize(ctx.stream));
    std::vector<double> Lz((size_t)n * n), zdev((size_t)n * nr);
    CK(hipMemcpy(Lz.data(), A, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(zdev.data(), fb + (size_t)n * nr, zdev.size() * 8, hipMemcpyDeviceToHost));
    double err = 0, zmax = 0;
    long bad = 0;
    for (int rr = 0; rr < nr; ++rr) {
      std::vector<double> z(n);
      for (int i = 0; i < n; ++i) {
        double v = (i < nreal && rr < nrhs) ? Yh[(size_t)i * nrhs + rr] - mean : 0.0;
        for (int k = 0; k < i; ++k) v -= Lz[(size_t)i * n + k] * z[k];
        z[i] = v / Lz[(size_t)i * n + i];
      }
      for (int i = 0; i < n; ++i) {
        const double dv = zdev[(size_t)i * nr + rr];
        if (!std::isfinite(dv)) ++bad;
        err = std::max(err, fabs(dv - z[i]));
        zmax = std::max(zmax, fabs(z[i]));
      }
    }
    printf("forward substitution nrhs=%d: z_done %d, max|z_dev - z_host| = %.3e (max|z| %.3e), non-finite %ld\n", nrhs,
           (int)zd, err, zmax, bad);
    CK(hipFree(Yd));
    CK(hipFree(fb));
  }
  // NOT_PD: a negative diagonal entry deep inside
  {
    std::vector<double> Kb = K;
    const int p = n / 2 + 37;
    Kb[(size_t)p * n + p] = -1.0;
    CK(hipMemcpy(A, Kb.data(), bytes, hipMemcpyHostToDevice));
    run(2, A, D, one);
    CK(hipStreamSynchronize(ctx.stream));
    CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
    int ref = 0;
    CK(hipMemcpy(A, Kb.data(), bytes, hipMemcpyHostToDevice));
    run(1, A, D, one);
    CK(hipStreamSynchronize(ctx.stream));
    CK(hipMemcpy(&ref, info, 4, hipMemcpyDeviceToHost));
    printf("NOT_PD at pivot %d: dag info %d, multi-launch info %d\n", p, hinfo, ref);
  }
  // timeout path: a tiny spin limit
  {
    ctx.spin_limit = 64;
    CK(hipMemcpy(A, K.data(), bytes, hipMemcpyHostToDevice));
    run(2, A, D, one);
    CK(hipStreamSynchronize(ctx.stream));
    CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
    printf("spin limit 64: info %d (INT_MIN = %d)\n", hinfo, INT_MIN);
    ctx.spin_limit = 1u << 22;
  }
  printf("DAG PROBE DONE\n");
  return 0;
}
