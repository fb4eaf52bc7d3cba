// Offline search for the band reductions' six-slab groups (actor-critic_amd/csrc/bandplan.hpp).
//
// The runtime planner is a greedy covering (fast, ~60% of the groups hold 9+ of
// their 16 sub-tile slots).  Blocks of unequal work drift apart in the image rows
// they stream, so the groups sharing a slab stop sharing it through L2; this
// search looks for an exact cover by FULL groups instead:
//   pool  = candidate six-slab sets (every 6-subset of the compact windows that
//           hold the needed pairs: 3x3 pixel windows for conv3, 4x2 slab windows
//           for conv2, and each dY slab with 5 slabs of its patch window(s));
//   flow  = every needed sub-tile assigned to one open set holding both its
//           slabs, at most 16 per set (bipartite b-matching, augmenting paths);
//   close = repeatedly close the least-loaded open set and re-route its tiles
//           through the remaining open sets; keep the closure when they all fit.
// Output: a C++ include with the groups (slab sets + assigned tile pairs),
// consumed by bandplan.hpp (band_plan_from_table) and checked at run time by
// acmi_selftest_plans (exact cover + host emulation of the fold).
//
//   g++ -O2 -std=c++17 -o /tmp/bps scripts/band_plan_search.cpp && /tmp/bps > actor-critic_amd/csrc/band_plans.inc
#include <algorithm>
#include <cmath>
#include <random>
#include <cstdio>
#include <deque>
#include <map>
#include <set>
#include <vector>

#include "../actor-critic_amd/csrc/bandplan.hpp"

using namespace acmi;

struct Search {
  int ns;
  std::vector<std::pair<int, int>> tiles;          // needed (a, b), a <= b
  std::vector<std::vector<int>> sets;              // candidate slab sets
  std::vector<std::vector<int>> tile_sets;         // tile -> candidate sets holding it
  std::vector<std::vector<int>> set_tiles;         // set -> tiles it could take
  std::vector<int> owner;                          // tile -> set
  std::vector<int> load;                           // set -> tiles assigned
  std::vector<char> open;
  int cap = 16;

  // augmenting path from tile t to an open set with spare capacity (BFS over
  // tiles; moving a tile frees a slot in the set it leaves)
  bool augment(int t0) {
    const int nt = (int)tiles.size();
    std::vector<int> prev_tile(nt, -2), via_set(nt, -1);
    std::deque<int> q;
    q.push_back(t0);
    prev_tile[t0] = -1;
    std::vector<char> seen_set(sets.size(), 0);
    while (!q.empty()) {
      const int t = q.front();
      q.pop_front();
      for (int s : tile_sets[t]) {
        if (!open[s] || seen_set[s] || s == owner[t]) continue;
        seen_set[s] = 1;
        if (load[s] < cap) {  // found: shift along the path
          int cur = t, tgt = s;
          ++load[tgt];
          while (cur >= 0) {
            const int old = owner[cur];
            owner[cur] = tgt;
            if (prev_tile[cur] < 0) {
              if (old >= 0) --load[old];
              break;
            }
            tgt = old;  // the previous tile moves into the set this one left
            cur = prev_tile[cur];
          }
          return true;
        }
        for (int u : set_tiles[s])
          if (owner[u] == s && prev_tile[u] == -2) {
            prev_tile[u] = t;
            q.push_back(u);
          }
      }
    }
    return false;
  }
};

static void emit(const char* name, const BandGeom& g, const Search& S) {
  // group layout: slabs of the set (sorted), tiles as slab-index pairs
  std::vector<int> used;
  for (size_t s = 0; s < S.sets.size(); ++s)
    if (S.open[s] && S.load[s] > 0) used.push_back((int)s);
  int units = 0;
  for (int s : used) units += (S.load[s] + 3) / 4;
  std::printf("// %s: %zu groups, %zu sub-tiles, sum of busiest-SIMD sub-tiles %d\n", name, used.size(),
              S.tiles.size(), units);
  std::printf("static const short %s_geom[7] = {%d, %d, %d, %d, %d, %d, %d};\n", name, g.H, g.W, g.C, g.KH,
              g.KW, g.S, g.CO);
  std::printf("static const short %s[][6 + 1 + 32] = {\n", name);
  for (int s : used) {
    std::vector<int> sl = S.sets[s];
    std::sort(sl.begin(), sl.end());
    std::printf("  {");
    for (int i = 0; i < 6; ++i) std::printf("%d, ", i < (int)sl.size() ? sl[i] : -1);
    std::printf("%d,", S.load[s]);
    int n = 0;
    for (size_t t = 0; t < S.tiles.size(); ++t)
      if (S.owner[t] == s) {
        std::printf(" %d, %d,", S.tiles[t].first, S.tiles[t].second);
        ++n;
      }
    for (; n < 16; ++n) std::printf(" -1, -1,");
    std::printf("},\n");
  }
  std::printf("};\n\n");
}

static long long argc_iters = 20000000LL;
static double argc_t0 = 3.0;
static unsigned argc_seed = 4242;
static void run(const char* name, int H, int W, int C, int KH, int KW, int S_, int CO) {
  BandGeom g;
  band_geom(H, W, C, KH, KW, S_, CO, &g);
  const std::vector<char> need = band_needed(g);
  Search S;
  S.ns = g.ns;
  std::map<std::pair<int, int>, int> tid;
  for (int a = 0; a < g.ns; ++a)
    for (int b = a; b < g.ns; ++b)
      if (need[(size_t)a * g.ns + b]) {
        tid[{a, b}] = (int)S.tiles.size();
        S.tiles.push_back({a, b});
      }
  // candidate pool
  std::set<std::vector<int>> pool;
  auto add_subsets = [&](const std::vector<int>& win, int k, std::vector<int> fixed) {
    const int n = (int)win.size();
    if (n < k) return;
    std::vector<int> idx(k);
    for (int i = 0; i < k; ++i) idx[i] = i;
    while (true) {
      std::vector<int> s = fixed;
      for (int i : idx) s.push_back(win[i]);
      std::sort(s.begin(), s.end());
      s.erase(std::unique(s.begin(), s.end()), s.end());
      if ((int)s.size() == (int)fixed.size() + k) pool.insert(s);
      int i = k - 1;
      while (i >= 0 && idx[i] == n - k + i) --i;
      if (i < 0) break;
      ++idx[i];
      for (int j = i + 1; j < k; ++j) idx[j] = idx[j - 1] + 1;
    }
  };
  // X windows: rows wy x slab columns wx (conv3: 3x3 pixels; conv2: 4 rows x 2 slab columns)
  const int sw = W / g.spx;  // slab columns
  const int wy = C == 64 ? 3 : 4, wx = C == 64 ? 3 : 2;
  for (int y0 = 0; y0 + wy <= H; ++y0)
    for (int x0 = 0; x0 + wx <= sw; ++x0) {
      std::vector<int> win;
      for (int y = y0; y < y0 + wy; ++y)
        for (int x = x0; x < x0 + wx; ++x) win.push_back(y * sw + x);
      add_subsets(win, 6, {});
    }
  // dY slabs with 5 slabs of each of their locations' patch windows
  for (int l = 0; l < g.L; ++l) {
    const int ly = l / g.OW, lx = l % g.OW;
    std::vector<int> win;
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw) win.push_back(band_xslab(g, S_ * ly + kh, S_ * lx + kw));
    std::sort(win.begin(), win.end());
    win.erase(std::unique(win.begin(), win.end()), win.end());
    add_subsets(win, 5, {band_yslab(g, l)});
  }
  for (const auto& s : pool) S.sets.push_back(s);
  const int ntile = (int)S.tiles.size(), nset = (int)S.sets.size();
  S.tile_sets.assign(ntile, {});
  S.set_tiles.assign(nset, {});
  for (int s = 0; s < nset; ++s) {
    const auto& v = S.sets[s];
    for (size_t i = 0; i < v.size(); ++i)
      for (size_t j = i; j < v.size(); ++j) {
        auto it = tid.find({v[i], v[j]});
        if (it == tid.end()) continue;
        S.tile_sets[it->second].push_back(s);
        S.set_tiles[s].push_back(it->second);
      }
  }
  for (int t = 0; t < ntile; ++t)
    if (S.tile_sets[t].empty()) {
      std::fprintf(stderr, "%s: tile (%d, %d) in no candidate set\n", name, S.tiles[t].first, S.tiles[t].second);
      std::exit(1);
    }
  S.owner.assign(ntile, -1);
  S.load.assign(nset, 0);
  S.open.assign(nset, 1);
  for (int t = 0; t < ntile; ++t)
    if (!S.augment(t)) {
      std::fprintf(stderr, "%s: initial flow failed\n", name);
      std::exit(1);
    }
  // Simulated annealing on the assignment: maximise sum(load^2) (concentrates
  // the tiles into few full sets) under the 16-tile cap; a move re-assigns one
  // tile to another candidate set holding both its slabs.
  std::mt19937 rng(argc_seed);
  long long energy = 0;
  for (int s = 0; s < nset; ++s) energy += (long long)S.load[s] * S.load[s];
  const double T0 = argc_t0, T1 = 0.05;
  const long long iters = argc_iters;
  auto used = [&]() {
    int n = 0;
    for (int s = 0; s < nset; ++s) n += S.load[s] > 0;
    return n;
  };
  int best_used = used();
  std::vector<int> best_owner = S.owner, best_load = S.load;
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<int> nz;
  for (long long it = 0; it < iters; ++it) {
    const double T = T0 * std::pow(T1 / T0, (double)it / iters);
    const int t = (int)(rng() % ntile);
    const auto& cs = S.tile_sets[t];
    int s2 = cs[rng() % cs.size()];
    if (U01(rng) < 0.9) {  // mostly propose sets already in use
      nz.clear();
      for (int x : cs)
        if (S.load[x] > 0 && S.load[x] < S.cap) nz.push_back(x);
      if (!nz.empty()) s2 = nz[rng() % nz.size()];
    }
    const int s1 = S.owner[t];
    if (s2 == s1 || S.load[s2] >= S.cap) continue;
    const int d = 2 * (S.load[s2] - S.load[s1]) + 2;
    if (d >= 0 || U01(rng) < std::exp(d / T)) {
      S.owner[t] = s2;
      --S.load[s1];
      ++S.load[s2];
      energy += d;
    }
    if ((it & 0xFFFFF) == 0) {
      const int u = used();
      if (u < best_used) best_used = u, best_owner = S.owner, best_load = S.load;
    }
  }
  {
    const int u = used();
    if (u < best_used) best_used = u, best_owner = S.owner, best_load = S.load;
  }
  S.owner = best_owner;
  S.load = best_load;
  std::fprintf(stderr, "%s: %d sets used (%d tiles)\n", name, best_used, ntile);
  emit(name, g, S);
}

int main(int argc, char** argv) {
  if (argc > 1) argc_iters = atoll(argv[1]);
  if (argc > 2) argc_t0 = atof(argv[2]);
  if (argc > 3) argc_seed = (unsigned)atoi(argv[3]);
  std::printf("// Generated by scripts/band_plan_search.cpp -- six-slab groups of the band\n");
  std::printf("// reductions: per group 6 slab ids, the tile count, then up to 16 (a, b) slab pairs.\n\n");
  run("kBandConv2", 20, 20, 32, 4, 4, 2, 64);
  run("kBandConv3c32", 9, 9, 64, 3, 3, 1, 32);
  run("kBandConv3c64", 9, 9, 64, 3, 3, 1, 64);
  return 0;
}
