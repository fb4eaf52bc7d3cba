// Host-side plan of the pixel-pair ("band") conv reductions (band.hpp).
//
// A conv layer's K-FAC input factor and weight gradient are sums over the M*L
// patch rows of [P;1]^T [P | dY].  Every product in them is a product of two
// INPUT PIXELS of one image (or of an input pixel and an output-gradient
// location), repeated once per patch that holds both.  The band reduction
// computes each such pixel-pair block once, over the M images:
//     T[a][b] = X_a^T X_b,   X = the input activations [M][H*W*C] (dense rows),
// for the 64-column slabs a, b of the row [X | dY] whose pixels share a patch,
// and folds the patch sums afterwards:  A[(k,c),(k',c')] = sum_l T[pix(l,k)][pix(l,k')][c][c'].
// conv3 (9x9x64 -> 7x7, 3x3 s1) needs 801 pixel-pair blocks instead of the
// 49 * 577^2/2 patch products per image: 2.5x fewer MACs; conv2 (20x20x32 -> 9x9,
// 4x4 s2): 1.6x fewer.  And the operand rows are dense runs instead of an
// im2col gather.
//
// This header is pure C++ (no HIP): the plan -- which 64x64 sub-tiles of the
// [X | dY]^T [X | dY] product are needed, grouped six slabs at a time for
// symred6_kernel (symred3.hpp), and the fold tables -- is built once per layer
// shape and checked by acmi_selftest_plans.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <random>
#include <vector>

namespace acmi {

struct BandGeom {
  int H, W, C;     // input image (NHWC), C in {32, 64}
  int KH, KW, S;   // VALID conv
  int CO;          // output channels, 64 % CO == 0 or CO == 64
  int OH, OW, L;   // output extent
  int spx;         // pixels per 64-column slab (64 / C)
  int nxs, nys;    // X slabs, dY slabs
  int ns;          // all slabs
  int kp;          // X columns (H*W*C)
  int J;           // X + dY columns
  int KK;          // kernel positions
};

inline bool band_geom(int H, int W, int C, int KH, int KW, int S, int CO, BandGeom* g) {
  if ((C != 32 && C != 64) || (CO != 32 && CO != 64) || W % (64 / C) != 0) return false;
  g->H = H, g->W = W, g->C = C, g->KH = KH, g->KW = KW, g->S = S, g->CO = CO;
  g->OH = (H - KH) / S + 1;
  g->OW = (W - KW) / S + 1;
  g->L = g->OH * g->OW;
  g->spx = 64 / C;
  g->nxs = H * W / g->spx;
  g->nys = (g->L * CO + 63) / 64;
  g->ns = g->nxs + g->nys;
  g->kp = H * W * C;
  g->J = g->kp + g->L * CO;
  g->KK = KH * KW;
  return true;
}

// pixel (y, x) -> slab and column offset inside it
inline int band_xslab(const BandGeom& g, int y, int x) { return (y * g.W + x) / g.spx; }
inline int band_xoff(const BandGeom& g, int x) { return (x % g.spx) * g.C; }
// output location l -> dY slab and column offset
inline int band_yslab(const BandGeom& g, int l) { return g.nxs + (l * g.CO) / 64; }
inline int band_yoff(const BandGeom& g, int l) { return (l * g.CO) % 64; }

// One work item of band_kernel (band.hpp): up to kBandSlabs staged 64-column
// slabs of [X | dY] (a prefix of `base`, nslab of them), up to two 64x64
// sub-tiles per wave (ra/cb index the staged slabs; -1: none), each with its
// compact tile id; csown: the staged slabs whose column sums this group writes
// (each slab's by exactly one group); xmask: bit i set when staged slab i is an
// X (layer input) slab -- its operand scale is the X scale, else the dY scale.
constexpr int kBandSlabs = 8;
struct BandGroup {
  int base[kBandSlabs];  // first [X | dY] column of each staged slab
  signed char ra[8][2];
  signed char cb[8][2];
  short tile[8][2];
  unsigned char csown;
  unsigned char nslab;
  unsigned char xmask;
  unsigned char pad;
};

struct BandPlan {
  BandGeom geom;
  std::vector<BandGroup> groups;
  // work lists per XCD: groups of one spatial region of the image (so an XCD's
  // L2 holds the columns its blocks stream), balanced by SIMD units
  std::vector<int> xcd_groups[8];
  int ntiles = 0;
  std::vector<int> tile_of;   // [ns * ns] (a <= b) -> tile id, -1 if not computed
  // fold tables: element offsets into the tile array T[ntiles][64][64] and the
  // column sums cs[ns * 64]
  std::vector<int> pairs;     // (ka, kb) kernel-position pairs in source orientation
  std::vector<int> atab;      // [npairs][L]: tile * 4096 + rowoff * 64 + coloff
  std::vector<int> wtab;      // [KK][L]: weight gradient source (X row slab, dY column slab)
  std::vector<int> ctab;      // [KK][L]: X column-sum column of pix(l, k)
  std::vector<int> dtab;      // [L]: dY column-sum column of location l
};

// the needed (a <= b) slab pairs of a layer
inline std::vector<char> band_needed(const BandGeom& g) {
  std::vector<char> need((size_t)g.ns * g.ns, 0);
  std::vector<int> sx;
  for (int ly = 0; ly < g.OH; ++ly)
    for (int lx = 0; lx < g.OW; ++lx) {
      sx.clear();
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw) sx.push_back(band_xslab(g, g.S * ly + kh, g.S * lx + kw));
      std::sort(sx.begin(), sx.end());
      sx.erase(std::unique(sx.begin(), sx.end()), sx.end());
      const int dl = band_yslab(g, ly * g.OW + lx);
      for (size_t i = 0; i < sx.size(); ++i) {
        for (size_t j = i; j < sx.size(); ++j) need[(size_t)sx[i] * g.ns + sx[j]] = 1;
        need[(size_t)sx[i] * g.ns + dl] = 1;
      }
    }
  return need;
}

// A group from its tiles: the staged slabs are the ones the tiles use, in column
// order; tile m goes to wave m % 8, slot m / 8 (waves w and w + 4 share a SIMD,
// so 13..16 tiles give every SIMD 3..4 sub-tiles)
inline BandGroup band_group_of(const BandGeom& g, const std::vector<std::pair<int, int>>& tiles) {
  std::vector<int> used;
  for (const auto& t : tiles) used.push_back(t.first), used.push_back(t.second);
  std::sort(used.begin(), used.end());
  used.erase(std::unique(used.begin(), used.end()), used.end());
  BandGroup G;
  G.nslab = (unsigned char)used.size();
  G.xmask = 0;
  for (int i = 0; i < kBandSlabs; ++i) {
    G.base[i] = i < (int)used.size() ? 64 * used[i] : -1;
    if (i < (int)used.size() && used[i] < g.nxs) G.xmask |= (unsigned char)(1u << i);
  }
  for (int w = 0; w < 8; ++w)
    for (int t = 0; t < 2; ++t) G.ra[w][t] = G.cb[w][t] = -1, G.tile[w][t] = -1;
  G.csown = 0;
  G.pad = 0;
  auto idx = [&](int slab) { return (int)(std::lower_bound(used.begin(), used.end(), slab) - used.begin()); };
  for (int m = 0; m < (int)tiles.size(); ++m) {
    G.ra[m % 8][m / 8] = (signed char)idx(tiles[m].first);
    G.cb[m % 8][m / 8] = (signed char)idx(tiles[m].second);
  }
  return G;
}

// Repair pass over a covering (off by default: modelled by scripts/band_l2sim.cpp,
// conv2's fabric bytes 2.44 -> 2.36 GB only): the greedy leaves a tail of small groups (conv2:
// 19 one-tile groups), whose blocks stream the image rows at a different pace
// from the full groups beside them, so the rows one block pulls into its XCD's
// L2 are gone when the others reach them.  Move every tile of the smallest
// groups into the fullest group that has a free slot and holds its slabs (or can
// stage the missing ones within NS); a group emptied this way is dropped.
inline void band_plan_repair(std::vector<std::vector<std::pair<int, int>>>& groups, int NS, int cap) {
  auto slabs_of = [](const std::vector<std::pair<int, int>>& gt) {
    std::vector<int> u;
    for (const auto& t : gt) u.push_back(t.first), u.push_back(t.second);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    return u;
  };
  for (int pass = 0; pass < 4; ++pass) {
    std::vector<int> ord(groups.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return groups[x].size() < groups[y].size(); });
    bool moved_any = false;
    for (int si : ord) {
      auto& src = groups[si];
      if (src.empty() || (int)src.size() >= 13) continue;
      // try to empty this group entirely: plan all moves first
      std::vector<std::vector<std::pair<int, int>>> trial = groups;
      bool ok = true;
      for (const auto& t : src) {
        int best = -1;
        for (size_t gi = 0; gi < trial.size(); ++gi) {
          if ((int)gi == si || trial[gi].empty() || (int)trial[gi].size() >= cap) continue;
          std::vector<int> u = slabs_of(trial[gi]);
          u.push_back(t.first), u.push_back(t.second);
          std::sort(u.begin(), u.end());
          u.erase(std::unique(u.begin(), u.end()), u.end());
          if ((int)u.size() > NS) continue;
          if (best < 0 || trial[gi].size() > trial[best].size()) best = (int)gi;
        }
        if (best < 0) {
          ok = false;
          break;
        }
        trial[best].push_back(t);
      }
      if (!ok) continue;
      trial[si].clear();
      groups.swap(trial);
      moved_any = true;
    }
    groups.erase(std::remove_if(groups.begin(), groups.end(), [](const auto& gt) { return gt.empty(); }),
                 groups.end());
    if (!moved_any) break;
  }
}

// Greedy covering of the needed sub-tiles by groups of <= kBandSlabs slabs and
// <= 16 tiles (two per wave): each of the 32 slabs with the most uncovered tiles
// seeds a candidate set grown by the neighbour adding the most uncovered tiles;
// the candidate with the most tiles (capped at 16; ties: fewest left over) wins
// and takes its 16 hardest tiles (fewest other uncovered tiles on their slabs).
// A group stages only the slabs its tiles use (the greedy's leftover groups are
// small).  Seeded restarts, the fewest groups kept.  Conv2 (M = 10240): 190
// groups, 117 of them full, against 243 six-slab groups of 9.5 tiles -- 8 slabs
// double the pairs a staged set can hold (28 + 8 against 15 + 6).
inline bool band_plan_build(const BandGeom& g, BandPlan* out, int restarts = 3, bool repair = false) {
  constexpr int NS = kBandSlabs;
  constexpr int cap = 16;
  const int ns = g.ns;
  const std::vector<char> need0 = band_needed(g);
  bool found = false;
  for (int rs = 0; rs < restarts; ++rs) {
    std::mt19937 rng(777u + rs);
    std::vector<char> need = need0;
    auto nd = [&](int x, int y) -> int {
      return x <= y ? need[(size_t)x * ns + y] : need[(size_t)y * ns + x];
    };
    std::vector<int> deg(ns, 0);
    std::vector<std::vector<int>> nbr(ns);
    int remaining = 0;
    for (int a = 0; a < ns; ++a)
      for (int b = a; b < ns; ++b)
        if (need[(size_t)a * ns + b]) {
          ++remaining;
          ++deg[a];
          if (b != a) ++deg[b], nbr[a].push_back(b), nbr[b].push_back(a);
        }
    std::vector<std::vector<std::pair<int, int>>> groups;  // each group's tiles (a <= b slabs)
    std::vector<int> order(ns);
    for (int i = 0; i < ns; ++i) order[i] = i;
    std::vector<int> cand;
    auto grow = [&](int s0, int* set) {
      int n = 0;
      set[n++] = s0;
      while (n < NS) {
        cand.clear();
        for (int i = 0; i < n; ++i)
          for (int y : nbr[set[i]])
            if (nd(set[i], y)) cand.push_back(y);
        if (cand.empty())  // nothing adjacent left: any slab with work
          for (int x : order)
            if (deg[x] > 0) cand.push_back(x);
        std::shuffle(cand.begin(), cand.end(), rng);
        int bx = -1, bg = -1;
        for (int x : cand) {
          bool in = false;
          for (int i = 0; i < n; ++i) in |= set[i] == x;
          if (in) continue;
          int gain = nd(x, x);
          for (int i = 0; i < n; ++i) gain += nd(x, set[i]);
          if (gain > bg) bg = gain, bx = x;
        }
        if (bx < 0) {  // fill with any other slab (dropped again below if unused)
          for (int x = 0; x < ns && bx < 0; ++x) {
            bool in = false;
            for (int i = 0; i < n; ++i) in |= set[i] == x;
            if (!in) bx = x;
          }
        }
        set[n++] = bx;
      }
      int tot = 0;
      for (int i = 0; i < NS; ++i)
        for (int j = i; j < NS; ++j) tot += nd(set[i], set[j]);
      return tot;
    };
    while (remaining > 0) {
      std::shuffle(order.begin(), order.end(), rng);
      int set[NS], best_key = -1, best_tot = 0;
      std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return deg[x] > deg[y]; });
      constexpr int kSeeds = 32;
      int tried = 0;
      for (int s0 : order) {
        if (deg[s0] == 0 || tried++ == kSeeds) break;
        int cs[NS];
        const int tot = grow(s0, cs);
        const int key = std::min(cap, tot);
        if (key > best_key || (key == best_key && tot < best_tot)) {
          best_key = key, best_tot = tot;
          for (int i = 0; i < NS; ++i) set[i] = cs[i];
        }
      }
      struct T {
        int a, b, key;
      };
      std::vector<T> tiles;
      for (int i = 0; i < NS; ++i)
        for (int j = i; j < NS; ++j) {
          const int a = std::min(set[i], set[j]), b = std::max(set[i], set[j]);
          if (nd(a, b)) tiles.push_back({a, b, deg[a] + deg[b]});
        }
      std::stable_sort(tiles.begin(), tiles.end(), [](const T& x, const T& y) { return x.key < y.key; });
      if ((int)tiles.size() > cap) tiles.resize(cap);
      std::vector<std::pair<int, int>> gt;
      for (const T& t : tiles) {
        need[(size_t)t.a * ns + t.b] = 0;
        --remaining;
        --deg[t.a];
        if (t.b != t.a) --deg[t.b];
        gt.push_back({t.a, t.b});
      }
      groups.push_back(gt);
    }
    if (repair) band_plan_repair(groups, NS, cap);
    if (found && groups.size() >= out->groups.size()) continue;
    out->geom = g;
    out->groups.clear();
    for (const auto& gt : groups) out->groups.push_back(band_group_of(g, gt));
    found = true;
  }
  if (!found) return false;
  BandPlan& p = *out;
  // spatial order (the image row a group's slabs sit on; dY slabs at the input
  // row their patch starts from), then 8 contiguous regions of equal SIMD work
  auto row_of = [&](int slab) -> double {
    if (slab < g.nxs) return (double)((slab * g.spx) / g.W);
    const int l = ((slab - g.nxs) * 64) / g.CO;
    return (double)(g.S * (l / g.OW)) + 0.5 * (g.KH - 1);
  };
  auto units = [](const BandGroup& G) {
    int u = 0;
    for (int w = 0; w < 4; ++w) {
      int t = 0;
      for (int h = 0; h < 2; ++h) t += (G.ra[w + 4 * h][0] >= 0) + (G.ra[w + 4 * h][1] >= 0);
      u = std::max(u, t);
    }
    return u;
  };
  std::vector<double> key(p.groups.size());
  for (size_t i = 0; i < p.groups.size(); ++i) {
    double k = 0;
    for (int j = 0; j < p.groups[i].nslab; ++j) k += row_of(p.groups[i].base[j] / 64);
    key[i] = k / std::max(1, (int)p.groups[i].nslab);
  }
  std::vector<int> ord(p.groups.size());
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return key[x] < key[y]; });
  {
    std::vector<BandGroup> sorted;
    for (int i : ord) sorted.push_back(p.groups[i]);
    p.groups.swap(sorted);
  }
  // work of a group: its busiest SIMD's sub-tiles + the staging it pays per slab
  auto work = [&](const BandGroup& G) { return 4.0 * units(G) + 0.5 * G.nslab + 1.0; };
  double total = 0;
  for (const BandGroup& G : p.groups) total += work(G);
  double acc = 0;
  for (int x = 0; x < 8; ++x) p.xcd_groups[x].clear();
  for (size_t i = 0; i < p.groups.size(); ++i) {
    const int x = std::min(7, (int)(8.0 * (acc + 0.5 * work(p.groups[i])) / total));
    p.xcd_groups[x].push_back((int)i);
    acc += work(p.groups[i]);
  }
  // within a region, the groups with the most sub-tiles first (spatial order among
  // equals): the blocks an XCD runs side by side then advance through the chunk's
  // rows at about the same pace, so the rows one of them pulls into L2 are still
  // there when the others reach them (conv2 band 0.654 -> 0.602 ms per launch)
  auto ntile = [&](int gi) {
    int t = 0;
    for (int w = 0; w < 8; ++w) t += (p.groups[gi].ra[w][0] >= 0) + (p.groups[gi].ra[w][1] >= 0);
    return t;
  };
  for (int x = 0; x < 8; ++x)
    std::stable_sort(p.xcd_groups[x].begin(), p.xcd_groups[x].end(),
                     [&](int a, int b) { return ntile(a) > ntile(b); });
  // tile ids (group-major), column-sum owners (first group staging the slab)
  p.tile_of.assign((size_t)ns * ns, -1);
  std::vector<char> csdone(ns, 0);
  int nt = 0;
  for (BandGroup& G : p.groups) {
    for (int w = 0; w < 8; ++w)
      for (int t = 0; t < 2; ++t) {
        if (G.ra[w][t] < 0) continue;
        const int a = G.base[G.ra[w][t]] / 64, b = G.base[G.cb[w][t]] / 64;
        G.tile[w][t] = (short)nt;
        p.tile_of[(size_t)a * ns + b] = nt++;
      }
    for (int i = 0; i < G.nslab; ++i) {
      const int s = G.base[i] / 64;
      if (!csdone[s]) csdone[s] = 1, G.csown |= (unsigned char)(1u << i);
    }
  }
  p.ntiles = nt;
  for (int s = 0; s < ns; ++s)
    if (!csdone[s]) return false;
  // fold tables
  auto pix_slab = [&](int l, int k, int* off) {
    const int ly = l / g.OW, lx = l % g.OW, kh = k / g.KW, kw = k % g.KW;
    const int y = g.S * ly + kh, x = g.S * lx + kw;
    *off = band_xoff(g, x);
    return band_xslab(g, y, x);
  };
  p.pairs.clear();
  p.atab.clear();
  for (int k1 = 0; k1 < g.KK; ++k1)
    for (int k2 = k1; k2 < g.KK; ++k2) {
      int o1, o2;
      const int s1 = pix_slab(0, k1, &o1), s2 = pix_slab(0, k2, &o2);
      const bool swap = s1 > s2;  // the slab order of the pair is the same at every l
      const int ka = swap ? k2 : k1, kb = swap ? k1 : k2;
      p.pairs.push_back(ka * 256 + kb);
      for (int l = 0; l < g.L; ++l) {
        int oa, ob;
        const int sa = pix_slab(l, ka, &oa), sb = pix_slab(l, kb, &ob);
        if (sa > sb) return false;
        const int t = p.tile_of[(size_t)sa * ns + sb];
        if (t < 0) return false;
        p.atab.push_back(t * 4096 + oa * 64 + ob);
      }
    }
  p.wtab.assign((size_t)g.KK * g.L, 0);
  p.ctab.assign((size_t)g.KK * g.L, 0);
  p.dtab.assign(g.L, 0);
  for (int k = 0; k < g.KK; ++k)
    for (int l = 0; l < g.L; ++l) {
      int o;
      const int s = pix_slab(l, k, &o), d = band_yslab(g, l);
      const int t = p.tile_of[(size_t)s * ns + d];
      if (t < 0) return false;
      p.wtab[(size_t)k * g.L + l] = t * 4096 + o * 64 + band_yoff(g, l);
      p.ctab[(size_t)k * g.L + l] = 64 * s + o;
    }
  for (int l = 0; l < g.L; ++l) p.dtab[l] = 64 * band_yslab(g, l) + band_yoff(g, l);
  return true;
}

// Coverage check (acmi_selftest_plans): every needed pair computed exactly once,
// at most two tiles per wave with slot 0 filled first, tiles only on staged
// slabs (a prefix of base, in column order), X/dY scale mask right, every slab's
// column sums owned once, every group in exactly one XCD list.
inline int band_plan_check(const BandPlan& p) {
  const BandGeom& g = p.geom;
  const std::vector<char> need = band_needed(g);
  std::vector<int> cov((size_t)g.ns * g.ns, 0), cs(g.ns, 0);
  for (const BandGroup& G : p.groups) {
    if (G.nslab < 1 || G.nslab > kBandSlabs) return 6;
    for (int i = 0; i < kBandSlabs; ++i) {
      if ((i < G.nslab) != (G.base[i] >= 0)) return 7;
      if (i > 0 && i < G.nslab && G.base[i] <= G.base[i - 1]) return 7;
      if (i < G.nslab && (((G.xmask >> i) & 1) != (G.base[i] / 64 < g.nxs))) return 8;
    }
    for (int w = 0; w < 8; ++w) {
      if (G.ra[w][0] < 0 && G.ra[w][1] >= 0) return 1;
      for (int t = 0; t < 2; ++t) {
        if (G.ra[w][t] < 0) continue;
        if (G.ra[w][t] >= G.nslab || G.cb[w][t] >= G.nslab) return 9;
        const int a = G.base[G.ra[w][t]] / 64, b = G.base[G.cb[w][t]] / 64;
        if (a > b || a >= g.nxs) return 2;
        cov[(size_t)a * g.ns + b]++;
      }
    }
    for (int i = 0; i < G.nslab; ++i)
      if (G.csown >> i & 1) cs[G.base[i] / 64]++;
  }
  for (size_t e = 0; e < need.size(); ++e)
    if (need[e] && cov[e] != 1) return 4;
  for (int s = 0; s < g.ns; ++s)
    if (cs[s] != 1) return 5;
  std::vector<int> seen(p.groups.size(), 0);
  for (int x = 0; x < 8; ++x)
    for (int i : p.xcd_groups[x]) {
      if (i < 0 || i >= (int)p.groups.size()) return 10;
      seen[i]++;
    }
  for (int v : seen)
    if (v != 1) return 10;
  return 0;
}

// Host emulation of the whole band path on M small pseudo-random images
// (double): the needed tiles of [X | dY]^T [X | dY] as the kernel stores them,
// the column sums, then the fold exactly as band_fold_kernel indexes its
// tables, against the direct patch-row definition [P;1]^T [P;1] / (M*L) and
// [P;1]^T dY.  Returns the largest relative deviation (~1e-16 when the plan and
// the tables are right).
inline double band_plan_emulate(const BandPlan& p, int M = 2) {
  const BandGeom& g = p.geom;
  const int ncol = g.ns * 64, K = g.KK * g.C, K1 = K + 1;
  std::mt19937 rng(99);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::vector<double> rows((size_t)M * ncol, 0.0);
  for (int m = 0; m < M; ++m)
    for (int c = 0; c < g.J; ++c) rows[(size_t)m * ncol + c] = U(rng);
  // kernel: tiles and column sums
  std::vector<double> T((size_t)p.ntiles * 4096, 0.0), cs(ncol, 0.0);
  for (int a = 0; a < g.ns; ++a)
    for (int b = a; b < g.ns; ++b) {
      const int t = p.tile_of[(size_t)a * g.ns + b];
      if (t < 0) continue;
      for (int m = 0; m < M; ++m) {
        const double* r = &rows[(size_t)m * ncol];
        for (int i = 0; i < 64; ++i)
          for (int j = 0; j < 64; ++j) T[(size_t)t * 4096 + i * 64 + j] += r[64 * a + i] * r[64 * b + j];
      }
    }
  for (int m = 0; m < M; ++m)
    for (int c = 0; c < ncol; ++c) cs[c] += rows[(size_t)m * ncol + c];
  // fold (band_fold_kernel)
  const double inv = 1.0 / ((double)M * g.L);
  std::vector<double> A((size_t)K1 * K1, 0.0), G((size_t)K1 * g.CO, 0.0);
  for (size_t P = 0; P < p.pairs.size(); ++P) {
    const int ka = p.pairs[P] >> 8, kb = p.pairs[P] & 255;
    for (int i = 0; i < g.C; ++i)
      for (int j = 0; j < g.C; ++j) {
        if (ka == kb && i > j) continue;
        double s = 0.0;
        for (int l = 0; l < g.L; ++l) s += T[(size_t)p.atab[P * g.L + l] + i * 64 + j];
        const int a = ka * g.C + i, b = kb * g.C + j;
        A[(size_t)a * K1 + b] = A[(size_t)b * K1 + a] = s * inv;
      }
  }
  for (int k = 0; k < g.KK; ++k)
    for (int ci = 0; ci < g.C; ++ci) {
      for (int co = 0; co < g.CO; ++co) {
        double s = 0.0;
        for (int l = 0; l < g.L; ++l) s += T[(size_t)p.wtab[k * g.L + l] + ci * 64 + co];
        G[(size_t)(k * g.C + ci) * g.CO + co] = s;
      }
      double s = 0.0;
      for (int l = 0; l < g.L; ++l) s += cs[p.ctab[k * g.L + l] + ci];
      A[(size_t)(k * g.C + ci) * K1 + K] = A[(size_t)K * K1 + k * g.C + ci] = s * inv;
    }
  for (int co = 0; co < g.CO; ++co) {
    double s = 0.0;
    for (int l = 0; l < g.L; ++l) s += cs[p.dtab[l] + co];
    G[(size_t)K * g.CO + co] = s;
  }
  A[(size_t)K * K1 + K] = 1.0;
  // direct definition over patch rows
  std::vector<double> Ad((size_t)K1 * K1, 0.0), Gd((size_t)K1 * g.CO, 0.0), pr(K1);
  for (int m = 0; m < M; ++m)
    for (int l = 0; l < g.L; ++l) {
      const double* r = &rows[(size_t)m * ncol];
      const int ly = l / g.OW, lx = l % g.OW;
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw)
          for (int c = 0; c < g.C; ++c)
            pr[(kh * g.KW + kw) * g.C + c] = r[((g.S * ly + kh) * g.W + g.S * lx + kw) * g.C + c];
      pr[K] = 1.0;
      for (int a = 0; a < K1; ++a) {
        for (int b = 0; b < K1; ++b) Ad[(size_t)a * K1 + b] += pr[a] * pr[b] * inv;
        for (int co = 0; co < g.CO; ++co) Gd[(size_t)a * g.CO + co] += pr[a] * r[g.kp + l * g.CO + co];
      }
    }
  double worst = 0.0, scale = 1e-300;
  for (size_t e = 0; e < A.size(); ++e) scale = std::max(scale, std::abs(Ad[e]));
  for (size_t e = 0; e < A.size(); ++e) worst = std::max(worst, std::abs(A[e] - Ad[e]) / scale);
  scale = 1e-300;
  for (size_t e = 0; e < G.size(); ++e) scale = std::max(scale, std::abs(Gd[e]));
  for (size_t e = 0; e < G.size(); ++e) worst = std::max(worst, std::abs(G[e] - Gd[e]) / scale);
  return worst;
}

}  // namespace acmi
