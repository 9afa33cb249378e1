// CPU check of the dataflow Cholesky's task lists (tools/, no GPU): for every list, a worst-case executor with P
// workers that take tasks strictly in list order and block on unmet dependencies must drain the graph, and every
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
  // two pools as on the device: F front workers take the front list [0, nfront), then join the bulk list
  const int F = plan.front_workers, nf = plan.nfront;
  int fnext = 0, bnext = nf;
  std::vector<int> held;  // tasks held by workers
  std::vector<int> hfront;  // workers still on the front list
  auto dec = [&](int q, int& type, int& a, int& b, int& k0, int& k1) {
    const unsigned long long c = plan.list[q];
    type = c & 0xff; a = (c >> 8) & 0xff; b = (c >> 16) & 0xff; k0 = (c >> 24) & 0xff; k1 = (c >> 32) & 0xff;
  };
  for (int iter = 0;; ++iter) {
    bool progress = false;
    // front workers (F of the P) hold front tasks while any remain; the rest hold bulk tasks
    {
      int nfront_held = 0;
      for (int q : held) nfront_held += q < nf;
      while ((int)held.size() < P) {
        const bool front_slot = nfront_held < F && fnext < nf;
        if (front_slot) { held.push_back(fnext); state[fnext++] = 1; ++nfront_held; progress = true; continue; }
        // a worker that is not holding a front task: bulk (front workers join once the front list is empty)
        const int bulk_workers = P - (fnext < nf ? F : nfront_held);
        int nbulk_held = (int)held.size() - nfront_held;
        if (bnext < nt && nbulk_held < bulk_workers) { held.push_back(bnext); state[bnext++] = 1; progress = true; continue; }
        break;
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
    for (size_t h = 0; h < held.size();) {
      const int q = held[h];
      int type, a, b, k0, k1;
      dec(q, type, a, b, k0, k1);
      bool done = false;
      if (type == T_FR) {
        const int i = a, k = b;
        int cols[3];
        const int nc = front_cols(k, nblk, cols);
        if (state[q] == 1) {
          bool ok = chain >= 2 * k + 2 && ver[i * nblk + k] >= k;
          for (int c2 = 0; c2 < nc; ++c2)
            if (cols[c2] <= i) ok = ok && ver[i * nblk + cols[c2]] >= k;
          if (ok) {
            if (ver[i * nblk + k] != k) { printf("FR(%d,%d) tile version %d\n", i, k, ver[i * nblk + k]); return false; }
            lrow[i] = k + 1;
            ver[i * nblk + k] = k + 1;  // L final
            state[q] = 3;                 // then the front blocks: 3 = diagonal pending, 4 + c2 = column c2 pending
            progress = true;
          }
        }
        if (state[q] == 3) {
          for (int c2 = 0; c2 < nc; ++c2)
            if (cols[c2] == i) {
              if (ver[i * nblk + i] != k) { printf("FR(%d,%d) diag version %d\n", i, k, ver[i * nblk + i]); return false; }
              ver[i * nblk + i] = k + 1;
            }
          state[q] = 4;
          progress = true;
        }
        while (state[q] >= 4 && state[q] - 4 < nc) {
          const int j = cols[state[q] - 4];
          if (j >= i) { ++state[q]; continue; }
          const bool lok = j == k + 1 ? cstep >= k + 2 : lrow[j] >= k + 1;
          if (!lok) break;
          if (ver[i * nblk + j] != k) { printf("FR(%d,%d) column %d version %d\n", i, k, j, ver[i * nblk + j]); return false; }
          ver[i * nblk + j] = k + 1;
          ++state[q];
          progress = true;
        }
        if (state[q] >= 4 && state[q] - 4 >= nc) done = true;
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
      if (done) { state[q] = 2; held[h] = held.back(); held.pop_back(); progress = true; }
      else ++h;
    }
    if (fnext >= nf && bnext >= nt && held.empty() && cstep >= nblk) break;
    if (!progress) { printf("DEADLOCK nblk=%d P=%d F=%d at front %d/%d bulk %d/%d chain step %d\n", nblk, P, F, fnext, nf, bnext, nt, cstep); return false; }
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
    printf("nblk=%d P=%d F=%d: %d tasks (FR %d, U64 %d, U128 %d), simulated %.1f us\n", nblk, P, plan.front_workers, (int)plan.list.size(), cnt[1], cnt[2], cnt[3], plan.sim_us);
  }
  return true;
}

int main() {
  bool ok = true;
  for (int nblk : {2, 4, 6, 8, 16, 32, 48, 64})
    for (int P : {7, 15, 31, 63, 127, 255}) ok = check(nblk, P, P == 255 || P == 63) && ok;
  for (int P : {255, 63}) {
    Plan pl = build_plan(64, P);
    printf("P=%d F=%d simulated chain starts:", P, pl.front_workers);
    for (size_t c = 0; c < pl.sim_chain.size(); c += 4) printf(" %.0f", pl.sim_chain[c]);
    printf("\n");
  }
  printf("%s\n", ok ? "PLAN CHECK OK" : "PLAN CHECK FAILED");
  return ok ? 0 : 1;
}
