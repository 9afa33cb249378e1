// CPU check of the dataflow Cholesky's task lists (tools/, no GPU): for every list, a worst-case executor with P
// workers that take tasks strictly in the order of their lists and block on unmet dependencies must drain the graph, and every
// 64-block must receive its stages exactly once, in order.  Also prints the simulated makespan.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gpx_potrf_dag.hip"
using namespace gpx::dag;

static bool check(int nblk, int P, bool verbose) {
  Plan plan = build_plan(nblk, P);
  std::vector<int> ver(nblk * nblk, 0), lrow(nblk, 0);
  int chain = 0;  // chain word
  const int nt = (int)plan.list.size();
  std::vector<int> state(nt, 0);  // 0 not taken, 1 taken (blocked or running), 2 done; FR: 3 = S part done
  int cstep = 0;
  // three pools as on the device: CW critical workers take [0, lend[0]), F front workers [lend[0], lend[1]); each
  // joins the bulk list [lend[1], lend[2]) once its own list is empty; the other workers take the bulk list
  const int CW = plan.crit_workers, F = plan.front_workers;
  int next[3] = {0, plan.lend[0], plan.lend[1]};
  struct Wk { int cls, held; };
  std::vector<Wk> wk(P);
  for (int p = 0; p < P; ++p) wk[p] = {p < CW ? 0 : (p < CW + F ? 1 : 2), -1};
  auto dec = [&](int q, int& type, int& a, int& b, int& k0, int& k1) {
    const unsigned long long c = plan.list[q];
    type = c & 0xff; a = (c >> 8) & 0xff; b = (c >> 16) & 0xff; k0 = (c >> 24) & 0xff; k1 = (c >> 32) & 0xff;
  };
  for (int iter = 0;; ++iter) {
    bool progress = false;
    for (Wk& w : wk) {
      while (w.held < 0) {
        if (next[w.cls] < plan.lend[w.cls]) {
          w.held = next[w.cls]++;
          state[w.held] = 1;
          progress = true;
        } else if (w.cls < 2) {
          w.cls = 2;
        } else {
          break;
        }
      }
    }
    // chain step
    if (cstep < nblk) {
      const bool ok = cstep == 0 || (ver[cstep * nblk + cstep - 1] >= cstep - 1 && ver[cstep * nblk + cstep] >= cstep - 1);
      if (ok) {
        if (cstep) {
          if (ver[cstep * nblk + cstep - 1] != cstep - 1 || ver[cstep * nblk + cstep] != cstep - 1) { printf("chain version mismatch\n"); return false; }
          ver[cstep * nblk + cstep - 1] = cstep;  // L_{c,c-1} final
          ver[cstep * nblk + cstep] = cstep;
        }
        chain = 2 * cstep + 2;
        ++cstep;
        progress = true;
      }
    }
    for (Wk& w : wk) {
      if (w.held < 0) continue;
      const int q = w.held;
      int type, a, b, k0, k1;
      dec(q, type, a, b, k0, k1);
      bool done = false;
      if (type == T_FR) {
        const int i = a, k = b;
        int order[kMaxFront];
        const int nord = fr_order(i, k, nblk, order);
        const bool crit = i == k + 2;
        if (state[q] == 1) {
          const bool pre = !crit || (ver[i * nblk + k + 1] >= k && ver[i * nblk + i] >= k);
          if (chain >= 2 * k + 2 && ver[i * nblk + k] >= k && pre) {
            if (ver[i * nblk + k] != k) { printf("FR(%d,%d) tile version %d\n", i, k, ver[i * nblk + k]); return false; }
            lrow[i] = k + 1;
            ver[i * nblk + k] = k + 1;  // L final
            state[q] = 4;               // 4 + q: front block order[q] pending
            progress = true;
          }
        }
        while (state[q] >= 4 && state[q] - 4 < nord) {
          const int j = order[state[q] - 4];
          if (ver[i * nblk + j] < k) break;
          if (j != i && !(j == k + 1 ? cstep >= k + 2 : lrow[j] >= k + 1)) break;
          if (ver[i * nblk + j] != k) { printf("FR(%d,%d) column %d version %d\n", i, k, j, ver[i * nblk + j]); return false; }
          ver[i * nblk + j] = k + 1;
          ++state[q];
          progress = true;
        }
        if (state[q] >= 4 && state[q] - 4 >= nord) done = true;
      } else {
        const int R = type == T_U64 ? 1 : 2;
        bool ok = true;
        for (int r = 0; r < R; ++r) ok = ok && lrow[R * a + r] >= k1 && lrow[R * b + r] >= k1;
        for (int r = 0; r < R; ++r)
          for (int s = 0; s < R; ++s)
            if (R * a + r >= R * b + s) ok = ok && ver[(R * a + r) * nblk + R * b + s] >= k0;
        if (ok) {
          for (int r = 0; r < R; ++r)
            for (int s = 0; s < R; ++s) {
              const int bi = R * a + r, bj = R * b + s;
              if (bi < bj) continue;
              if (ver[bi * nblk + bj] != k0) { printf("U%d(%d,%d,%d,%d) block (%d,%d) at version %d\n", 64 * R, a, b, k0, k1, bi, bj, ver[bi * nblk + bj]); return false; }
              ver[bi * nblk + bj] = k1;
            }
          done = true;
        }
      }
      if (done) { state[q] = 2; w.held = -1; progress = true; }
    }
    bool idle = cstep >= nblk;
    for (const Wk& w : wk) idle = idle && w.held < 0;
    for (int c = 0; c < 3; ++c) idle = idle && next[c] >= plan.lend[c];
    if (idle) break;
    if (!progress) { printf("DEADLOCK nblk=%d P=%d CW=%d F=%d at lists %d %d %d chain step %d\n", nblk, P, CW, F, next[0], next[1], next[2], cstep); return false; }
  }
  // every block (i, j), i > j: versions reach j + 1 (L final), diagonal: j
  for (int i = 0; i < nblk; ++i)
    for (int j = 0; j <= i; ++j) {
      const int want = i == j ? j : j + 1;
      if (ver[i * nblk + j] != want && !(i == j && ver[i * nblk + j] == j + 0)) {
        if (!(i == j)) { printf("block (%d,%d) final version %d, want %d\n", i, j, ver[i * nblk + j], want); return false; }
      }
    }
  if (verbose) {
    int cnt[4] = {0};
    for (auto c : plan.list) cnt[c & 0xff]++;
    printf("nblk=%d P=%d CW=%d F=%d: %d tasks (FR %d, U64 %d, U128 %d), simulated %.1f us\n", nblk, P, plan.crit_workers, plan.front_workers, (int)plan.list.size(), cnt[1], cnt[2], cnt[3], plan.sim_us);
  }
  return true;
}

int main() {
  bool ok = true;
  for (int nblk : {2, 4, 6, 8, 16, 32, 48, 64})
    for (int P : {7, 15, 31, 63, 127, 255}) ok = check(nblk, P, P == 255 || P == 63) && ok;
  for (int P : {255, 63}) {
    Plan pl = build_plan(64, P);
    printf("P=%d F=%d busy: front %.0f of %.0f, bulk %.0f of %.0f worker-us; chain starts:", P, pl.front_workers,
           pl.sim_busy_front, pl.front_workers * pl.sim_us, pl.sim_busy_bulk, (P - pl.front_workers) * pl.sim_us);
    for (size_t c = 0; c < pl.sim_chain.size(); c += 4) printf(" %.0f", pl.sim_chain[c]);
    printf("\n  critical FR(c+1,c-1) relative to chain step c start: taken, tiles final, L published, done | next step\n");
    for (size_t c = 2; c + 1 < pl.sim_chain.size(); c += (P == 255 ? 1 : 5)) {
      const double b = pl.sim_chain[c];
      const double* x = &pl.sim_crit[7 * (c - 1)];
      printf("  c=%2zu %7.1f %7.1f %7.1f %7.1f | %7.1f   tiles (c+1,c-1) %6.1f (c+1,c) %6.1f (c+1,c+1) %6.1f\n", c,
             x[0] - b, x[1] - b, x[2] - b, x[3] - b, pl.sim_chain[c + 1] - b, x[4] - b, x[5] - b, x[6] - b);
    }
  }
  printf("%s\n", ok ? "PLAN CHECK OK" : "PLAN CHECK FAILED");
  return ok ? 0 : 1;
}
