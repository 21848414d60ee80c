// Host model of cheb_fwd_fast's LDS bank conflicts on a graph's fast layout
// (lds_layout.cpp): for each LDS wave-instruction group of one workgroup's
// recurrence -- the gathers, the two own-record writes, the MFMA tile reads --
// the extra cycles max_bank(distinct addresses) - 1 per 32-lane half, by the
// bank rule of MI355X_MICROARCH.md §LDS ((a/4) mod 32 for ds_read_b32 and
// ds_write_b32).  Compared with SQ_LDS_BANK_CONFLICT of the ablation passes
// (scripts/gpu_r04_lds.sh).   lds_model M.bin rp.bin ci.bin K N
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#include "../../cnn_graph_amd/csrc/cg_internal.h"

static std::vector<int> rd(const char* p) {
  FILE* f = fopen(p, "rb");
  std::vector<int> v;
  int x;
  while (fread(&x, 4, 1, f) == 1) v.push_back(x);
  fclose(f);
  return v;
}

// extra cycles of one 32-lane group of byte addresses
static int extra(const std::vector<int>& addr) {
  std::map<int, std::set<int>> b;
  for (int a : addr) b[(a / 4) % 32].insert(a);
  size_t mx = 1;
  for (auto& kv : b) mx = std::max(mx, kv.second.size());
  return int(mx) - 1;
}

int main(int argc, char** argv) {
  const int M = rd(argv[1])[0];
  std::vector<int> rp = rd(argv[2]), ci = rd(argv[3]);
  const int K = atoi(argv[4]), N = atoi(argv[5]);
  cg::FastLayout lay;
  cg::plan_fast_layout(M, rp.data(), ci.data(), &lay);
  const int REC = 12, kT = 1024, kW = 16;
  long g_extra = 0, w_extra = 0, t_extra = 0, g_n = 0, w_n = 0, t_n = 0;
  for (int slot = 0; slot < 3; ++slot) {
    for (int w = 0; w < kW; ++w)
      for (int h = 0; h < 2; ++h) {
        const int l0 = w * 64 + h * 32;
        for (int j = 0; j < lay.wlen[w]; ++j) {
          std::vector<int> a;
          for (int i = 0; i < 32; ++i) a.push_back(lay.cpos[size_t(j) * kT + l0 + i] * REC + slot * 4);
          g_extra += extra(a);
          g_n++;
        }
        for (int c = 0; c < 2; ++c) {
          std::vector<int> a;
          for (int i = 0; i < 32; ++i)
            a.push_back((c ? lay.rpos1[l0 + i] : lay.rpos0[l0 + i]) * REC + slot * 4);
          w_extra += extra(a);
          w_n++;
        }
      }
    const int ntiles = (M + 31) / 32;
    for (int tl = 0; tl < ntiles; ++tl) {
      std::vector<int> a;
      for (int i = 0; i < 32; ++i) a.push_back(lay.mpos[size_t(tl) * 32 + i] * REC + slot * 4);
      t_extra += extra(a);
      t_n++;
    }
  }
  // per step: average over the 3 ring slots; K-1 steps; tile reads: every
  // pair (ceil(K/2)) two halves (slots of kk = 2s and 2s+1), wave-instruction
  // per tile of each wave
  const double steps = K - 1, pairs = (K + 1) / 2;
  const double g = g_extra / 3.0 * steps * N, wr = w_extra / 3.0 * steps * N;
  const double t = t_extra / 3.0 * 2 * pairs * N;
  printf("{\"M\": %d, \"K\": %d, \"N\": %d, \"gather_groups_per_step\": %.0f, \"gather_extra_per_step\": %.1f, "
         "\"write_groups_per_step\": %.0f, \"write_extra_per_step\": %.1f, \"tile_groups\": %.0f, "
         "\"tile_extra\": %.1f, \"dispatch_extra\": {\"gathers\": %.0f, \"writes\": %.0f, \"tiles\": %.0f}}\n",
         M, K, N, g_n / 3.0, g_extra / 3.0, w_n / 3.0, w_extra / 3.0, t_n / 3.0, t_extra / 3.0, g, wr, t);
  return 0;
}
