// Bank-aware LDS layout of the recurrence ring for the fast resident kernels
// (cheb_fast.hip).  Host code, run once per plan (cg_plan_create).
//
// Every Chebyshev step is one burst of ds_read_b32 gathers: wave-instruction j
// of wave w reads, for each of its 64 rows, the record of the row's j-th CSR
// column.  LDS serves a ds_read_b32 in two 32-lane groups, one cycle per group
// when the 32 addresses fall in 32 different banks ((addr/4) mod 32) and one
// more cycle for every extra distinct address in a bank.  With the vertex
// records in vertex order the MNIST graph's gathers take 2.7x the conflict-
// free cycles.  This module places the records so that they do not:
//   * every vertex has TWO records (copies) whose bank classes (position mod
//     32) are chosen independently; the owner of a row writes both copies each
//     step (one extra ds_write), and every gathering lane reads whichever copy
//     keeps its 32-lane group conflict-free;
//   * padding entries read one of 32 zero records (one per bank) and idle
//     lanes write one of 32 dummy records, so neither ever adds a conflict;
//   * bank classes are chosen by simulated annealing over the cost
//        sum over every LDS wave-instruction group of (max distinct addresses
//        in one bank)
//     covering the gathers, the T_{k-2} read, the two record writes and the
//     MFMA tile reads; the per-group copy choice is a greedy assignment with
//     improvement passes.  Fixed seed: the layout is a deterministic function
//     of the graph.
// Only WHERE values live changes; every row still accumulates its CSR entries
// in order, so results are bit-identical for every layout.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include <vector>

#include "cg_internal.h"

namespace cg {
namespace {

constexpr int kBanks = 32;
constexpr int kT = 1024;
constexpr int kW = kT / 64;

struct Item {
  int v;     // vertex (>= 0), or -1 = free (zero / dummy record: any bank)
};

struct Group {
  std::vector<int> verts;  // distinct vertices read/written by the group
  int nfree;               // lanes that may take any bank (pads / idle), deduplicated to <= 1 each
  int copy;                // -1: lanes choose a copy; 0/1: fixed copy (writes)
  float weight;
};

// augmenting paths of the b-matching in group_cost: vertex x into one of its
// two candidate banks of capacity cap, displacing (recursively) a vertex that
// can move to its other bank
struct Aug {
  const int (*cand)[2];
  int cap;
  int fill[kBanks] = {0};
  int slot[kBanks][64];
  bool vis[kBanks];
  bool run(int x, int* c2) {
    for (int e = 0; e < 2; ++e) {
      const int bk = cand[x][e];
      if (vis[bk]) continue;
      vis[bk] = true;
      if (fill[bk] < cap) {
        slot[bk][fill[bk]++] = x;
        c2[x] = e;
        return true;
      }
      for (int q = 0; q < fill[bk]; ++q) {
        const int y = slot[bk][q];
        if (run(y, c2)) {  // y moved to its other bank
          slot[bk][q] = x;
          c2[x] = e;
          return true;
        }
      }
    }
    return false;
  }
};

// Copy assignment for one group with the smallest max bank load (free lanes
// included): a greedy start, then, while the max load exceeds the lower bound,
// an exact check by augmenting paths whether every vertex fits in banks of
// capacity cap = bound, bound + 1, ... (each vertex has two candidate banks,
// so this is a bipartite b-matching).  Returns the max bank load.
int group_cost(const Group& g, const std::vector<int8_t>& b0, const std::vector<int8_t>& b1,
               int* choice /* may be null */) {
  const int n = int(g.verts.size());
  int cand[64][2];
  int nd = 0;  // distinct candidates
  for (int i = 0; i < n; ++i) {
    const int v = g.verts[size_t(i)];
    cand[i][0] = b0[size_t(v)];
    cand[i][1] = g.copy >= 0 ? (g.copy ? b1[size_t(v)] : b0[size_t(v)]) : b1[size_t(v)];
    if (g.copy == 1) cand[i][0] = cand[i][1];
    nd += cand[i][0] != cand[i][1];
  }
  int chs[64];
  int load[kBanks] = {0};
  for (int i = 0; i < n; ++i) {  // greedy
    const int c = load[cand[i][0]] <= load[cand[i][1]] ? 0 : 1;
    chs[i] = c;
    load[cand[i][c]]++;
  }
  auto finish = [&](int* ld) {
    for (int f = 0; f < g.nfree; ++f) {  // free lanes take the emptiest banks
      int best = 0;
      for (int b = 1; b < kBanks; ++b)
        if (ld[b] < ld[best]) best = b;
      ld[best]++;
    }
    int mx = 0;
    for (int b = 0; b < kBanks; ++b) mx = std::max(mx, ld[b]);
    return mx;
  };
  int tmp[kBanks];
  std::copy(load, load + kBanks, tmp);
  int best = finish(tmp);
  const int bound = (n + g.nfree + kBanks - 1) / kBanks;
  if (best > bound && nd > 0) {
    for (int cap = bound; cap < best; ++cap) {
      // b-matching of vertices to banks of capacity cap (free lanes fit when
      // some bank stays below cap, i.e. n + nfree <= 32 cap)
      if (n + g.nfree > kBanks * cap) continue;
      int c2[64];
      Aug m{cand, cap};
      bool ok = true;
      for (int i = 0; i < n && ok; ++i) {
        std::fill(m.vis, m.vis + kBanks, false);
        ok = m.run(i, c2);
      }
      if (!ok) continue;
      int ld[kBanks] = {0};
      for (int i = 0; i < n; ++i) ld[cand[i][c2[i]]]++;
      const int mx = finish(ld);
      if (mx < best) {
        best = mx;
        std::copy(c2, c2 + n, chs);
      }
      break;
    }
  }
  if (choice)
    for (int i = 0; i < n; ++i) choice[i] = g.copy >= 0 ? g.copy : chs[i];
  return best;
}

}  // namespace

// See cg_internal.h::FastLayout.
void plan_fast_layout(int M, const int32_t* rp, const int32_t* ci, FastLayout* out) {
  const int width = kFastWidth;
  // thread t -> row: decreasing length, stable
  std::vector<int> order(static_cast<size_t>(M));
  for (int r = 0; r < M; ++r) order[size_t(r)] = r;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return (rp[a + 1] - rp[a]) > (rp[b + 1] - rp[b]); });
  std::vector<int> trow(kT, -1);
  for (int t = 0; t < M; ++t) trow[size_t(t)] = order[size_t(t)];
  std::vector<int> wlen(kW, 0);
  for (int t = 0; t < M; ++t) {
    const int r = trow[size_t(t)];
    wlen[size_t(t / 64)] = std::max(wlen[size_t(t / 64)], rp[r + 1] - rp[r]);
  }

  // ---- groups ---------------------------------------------------------------
  std::vector<Group> groups;
  // gather groups: (wave, half, slot): lane (w*64 + h*32 + i) reads column j of its row
  std::vector<std::vector<int>> gather_gid(size_t(width), std::vector<int>(kT / 32, -1));
  for (int w = 0; w < kW; ++w)
    for (int h = 0; h < 2; ++h)
      for (int j = 0; j < wlen[size_t(w)]; ++j) {
        Group g;
        g.copy = -1;
        g.weight = 1.f;
        g.nfree = 0;
        bool pad = false;
        for (int i = 0; i < 32; ++i) {
          const int r = trow[size_t(w * 64 + h * 32 + i)];
          if (r >= 0 && j < rp[r + 1] - rp[r]) g.verts.push_back(ci[rp[r] + j]);
          else pad = true;
        }
        std::sort(g.verts.begin(), g.verts.end());
        g.verts.erase(std::unique(g.verts.begin(), g.verts.end()), g.verts.end());
        g.nfree = pad ? 1 : 0;
        gather_gid[size_t(j)][size_t(w * 2 + h)] = int(groups.size());
        groups.push_back(std::move(g));
      }
  // own-record groups per (wave, half): T_{k-2} read (choose copy), write copy 0, write copy 1
  std::vector<int> prv_gid(kT / 32, -1);
  for (int w = 0; w < kW; ++w)
    for (int h = 0; h < 2; ++h) {
      Group g;
      g.nfree = 0;
      for (int i = 0; i < 32; ++i) {
        const int r = trow[size_t(w * 64 + h * 32 + i)];
        if (r >= 0) g.verts.push_back(r);
        else g.nfree = 1;
      }
      if (g.verts.empty()) continue;
      g.weight = 1.f;
      g.copy = -1;
      prv_gid[size_t(w * 2 + h)] = int(groups.size());
      groups.push_back(g);
      g.copy = 0;
      groups.push_back(g);
      g.copy = 1;
      groups.push_back(g);
    }
  // MFMA tile reads: 32 consecutive vertices, every other step
  const int ntiles = (M + 31) / 32;
  std::vector<int> tile_gid(size_t(ntiles), -1);
  for (int tl = 0; tl < ntiles; ++tl) {
    Group g;
    g.copy = -1;
    g.weight = 0.5f;
    g.nfree = (tl * 32 + 32 > M) ? 1 : 0;
    for (int i = 0; i < 32 && tl * 32 + i < M; ++i) g.verts.push_back(tl * 32 + i);
    tile_gid[size_t(tl)] = int(groups.size());
    groups.push_back(std::move(g));
  }
  std::vector<std::vector<int>> vgroups(static_cast<size_t>(M));
  for (int gi = 0; gi < int(groups.size()); ++gi)
    for (int v : groups[size_t(gi)].verts) vgroups[size_t(v)].push_back(gi);

  // ---- annealing over bank classes ----------------------------------------------
  // The two own-record writes of a 32-lane half are conflict-free by
  // construction: within every half the rows' copy-0 classes are a set of
  // distinct banks, and so are their copy-1 classes, and the annealing moves
  // keep it so (swap two rows' classes of one copy inside a half, or move a
  // row to a class its half leaves unused).  The gathers and the MFMA tile
  // reads are what it optimises.
  std::vector<int8_t> b0(static_cast<size_t>(M)), b1(static_cast<size_t>(M));
  std::vector<int> half_of(static_cast<size_t>(M), -1);
  std::vector<std::vector<int>> half_rows(kT / 32);
  for (int t = 0; t < kT; ++t)
    if (trow[size_t(t)] >= 0) {
      half_of[size_t(trow[size_t(t)])] = t / 32;
      half_rows[size_t(t / 32)].push_back(trow[size_t(t)]);
    }
  std::mt19937 rng(20170u);
  for (auto& hr : half_rows) {
    int perm[kBanks];
    for (int b = 0; b < kBanks; ++b) perm[b] = b;
    std::shuffle(perm, perm + kBanks, rng);
    for (size_t i = 0; i < hr.size(); ++i) {
      b0[size_t(hr[i])] = int8_t(i);
      b1[size_t(hr[i])] = int8_t(perm[i]);
    }
  }
  std::vector<int> gc(groups.size());
  double total = 0;
  for (size_t gi = 0; gi < groups.size(); ++gi) {
    gc[gi] = group_cost(groups[gi], b0, b1, nullptr);
    total += groups[gi].weight * gc[gi];
  }
  const long iters = std::max<long>(400000, 400L * M);
  const double T0 = 1.0, T1 = 0.02;
  // stop early at the bound: every group at its fewest possible cycles
  double lower = 0;
  for (const Group& g : groups)
    lower += g.weight * ((int(g.verts.size()) + g.nfree + kBanks - 1) / kBanks);
  std::vector<int> aff, newc;
  for (long it = 0; it < iters && total > lower + 1e-6; ++it) {
    const double T = T0 * std::pow(T1 / T0, double(it) / double(iters));
    const int v = int(rng() % uint32_t(M));
    const int c = int(rng() & 1u);
    std::vector<int8_t>& b = c ? b1 : b0;
    const std::vector<int>& hr = half_rows[size_t(half_of[size_t(v)])];
    const int8_t nb = int8_t(rng() % kBanks);
    if (nb == b[size_t(v)]) continue;
    int u = -1;  // the half's row holding class nb (swapped with v), if any
    for (int x : hr)
      if (b[size_t(x)] == nb) u = x;
    const int8_t old = b[size_t(v)];
    b[size_t(v)] = nb;
    if (u >= 0) b[size_t(u)] = old;
    aff = vgroups[size_t(v)];
    if (u >= 0) aff.insert(aff.end(), vgroups[size_t(u)].begin(), vgroups[size_t(u)].end());
    std::sort(aff.begin(), aff.end());
    aff.erase(std::unique(aff.begin(), aff.end()), aff.end());
    newc.resize(aff.size());
    double d = 0;
    for (size_t q = 0; q < aff.size(); ++q) {
      const Group& g = groups[size_t(aff[q])];
      newc[q] = group_cost(g, b0, b1, nullptr);
      d += g.weight * (newc[q] - gc[size_t(aff[q])]);
    }
    const double uu = double(rng()) / 4294967296.0;
    if (d <= 0 || uu < std::exp(-d / T)) {
      for (size_t q = 0; q < aff.size(); ++q) gc[size_t(aff[q])] = newc[q];
      total += d;
    } else {
      b[size_t(v)] = old;
      if (u >= 0) b[size_t(u)] = nb;
    }
  }

  // ---- positions: record p has bank class p % 32 ----------------------------------
  // slot 0 of every class: zero record; slot 1: dummy record; vertex copies after.
  std::vector<int> fill(kBanks, 2);
  out->pos0.assign(size_t(M), 0);
  out->pos1.assign(size_t(M), 0);
  for (int v = 0; v < M; ++v) {
    const int c0 = b0[size_t(v)];
    out->pos0[size_t(v)] = c0 + kBanks * fill[size_t(c0)]++;
    const int c1 = b1[size_t(v)];
    out->pos1[size_t(v)] = c1 + kBanks * fill[size_t(c1)]++;
  }
  const int slots = *std::max_element(fill.begin(), fill.end());
  out->P = kBanks * slots;
  out->zero_base = 0;   // zero record of bank b: position b
  out->dummy_base = kBanks;

  // ---- per-thread image ---------------------------------------------------------
  out->row = trow;
  out->wlen = wlen;
  out->cpos.assign(size_t(width) * kT, 0);
  out->rpos0.assign(kT, 0);
  out->rpos1.assign(kT, 0);
  out->rposr.assign(kT, 0);
  auto position = [&](int v, int c) { return c ? out->pos1[size_t(v)] : out->pos0[size_t(v)]; };
  auto bank_of = [&](int p) { return p % kBanks; };
  // lanes of a group that take a free record pick a bank the group leaves empty
  auto free_banks = [&](const std::vector<int>& used_pos) {
    std::vector<int> load(kBanks, 0);
    for (int p : used_pos) load[size_t(bank_of(p))]++;
    int best = 0;
    for (int b = 1; b < kBanks; ++b)
      if (load[size_t(b)] < load[size_t(best)]) best = b;
    return best;
  };
  int choice[64];
  for (int w = 0; w < kW; ++w)
    for (int h = 0; h < 2; ++h) {
      const int lane0 = w * 64 + h * 32;
      for (int j = 0; j < wlen[size_t(w)]; ++j) {
        const Group& g = groups[size_t(gather_gid[size_t(j)][size_t(w * 2 + h)])];
        group_cost(g, b0, b1, choice);
        std::vector<int> used;
        for (size_t i = 0; i < g.verts.size(); ++i) used.push_back(position(g.verts[i], choice[i]));
        const int zb = free_banks(used);
        for (int i = 0; i < 32; ++i) {
          const int t = lane0 + i;
          const int r = trow[size_t(t)];
          int p = out->zero_base + zb;
          if (r >= 0 && j < rp[r + 1] - rp[r]) {
            const int v = ci[rp[r] + j];
            const size_t k = size_t(std::lower_bound(g.verts.begin(), g.verts.end(), v) - g.verts.begin());
            p = position(v, choice[k]);
          }
          out->cpos[size_t(j) * kT + t] = p;
        }
      }
      for (int j = wlen[size_t(w)]; j < width; ++j)
        for (int i = 0; i < 32; ++i) out->cpos[size_t(j) * kT + lane0 + i] = out->zero_base;
      // own records
      const int pg = prv_gid[size_t(w * 2 + h)];
      std::vector<int> used0, used1, usedr;
      if (pg >= 0) group_cost(groups[size_t(pg)], b0, b1, choice);
      int k = 0;
      for (int i = 0; i < 32; ++i) {
        const int r = trow[size_t(lane0 + i)];
        if (r < 0) continue;
        used0.push_back(out->pos0[size_t(r)]);
        used1.push_back(out->pos1[size_t(r)]);
        usedr.push_back(position(r, choice[k]));
        out->rpos0[size_t(lane0 + i)] = out->pos0[size_t(r)];
        out->rpos1[size_t(lane0 + i)] = out->pos1[size_t(r)];
        out->rposr[size_t(lane0 + i)] = position(r, choice[k]);
        ++k;
      }
      // idle lanes: dummy records in banks the active lanes' writes leave
      // empty, chosen per copy (both writes stay conflict-free)
      std::vector<int> load0(kBanks, 0), load1(kBanks, 0);
      for (int p : used0) load0[size_t(bank_of(p))]++;
      for (int p : used1) load1[size_t(bank_of(p))]++;
      auto emptiest = [&](std::vector<int>& ld) {
        int best = 0;
        for (int b = 1; b < kBanks; ++b)
          if (ld[size_t(b)] < ld[size_t(best)]) best = b;
        ld[size_t(best)]++;
        return best;
      };
      for (int i = 0; i < 32; ++i) {
        const int t = lane0 + i;
        if (trow[size_t(t)] >= 0) continue;
        out->rpos0[size_t(t)] = out->rposr[size_t(t)] = out->dummy_base + emptiest(load0);
        out->rpos1[size_t(t)] = out->dummy_base + emptiest(load1);
      }
    }
  // MFMA tile reads
  out->mpos.assign(size_t(ntiles) * 32, out->zero_base);
  for (int tl = 0; tl < ntiles; ++tl) {
    const Group& g = groups[size_t(tile_gid[size_t(tl)])];
    group_cost(g, b0, b1, choice);
    std::vector<int> used;
    for (size_t i = 0; i < g.verts.size(); ++i) {
      const int p = position(g.verts[i], choice[i]);
      used.push_back(p);
      out->mpos[size_t(tl) * 32 + i] = p;
    }
    const int zb = free_banks(used);
    for (int i = int(g.verts.size()); i < 32; ++i) out->mpos[size_t(tl) * 32 + size_t(i)] = zb;
  }
  // conflict statistics (for the ABI's introspection / tests)
  long gathers = 0, ideal = 0;
  for (int w = 0; w < kW; ++w)
    for (int h = 0; h < 2; ++h)
      for (int j = 0; j < wlen[size_t(w)]; ++j) {
        gathers += gc[size_t(gather_gid[size_t(j)][size_t(w * 2 + h)])];
        ideal += 1;
      }
  out->gather_cycles = gathers;
  out->gather_ideal = ideal;
}

}  // namespace cg
