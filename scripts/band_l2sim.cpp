// Offline model of the conv2 band kernel's L2 traffic (band.hpp / bandplan.hpp):
// 8 XCDs, 32 CUs each, one block per CU taking the XCD's work items in list
// order as CUs free up; every K-tile of an item touches its staged slabs' 16 rows
// (two 128-B lines per slab row); each XCD's 4 MiB L2 is an LRU over 128-B lines.
// Time per K-tile of an item = c0 + busiest SIMD's sub-tiles (units).  Prints
// the modelled hit rate and fabric bytes for the plan as built and for variants.
//   g++ -O2 -std=c++17 -o /tmp/l2sim scripts/band_l2sim.cpp && /tmp/l2sim
#include <cstdio>
#include <list>
#include <queue>
#include <unordered_map>
#include <vector>

#include "../actor-critic_amd/csrc/bandplan.hpp"

using namespace acmi;

struct LRU {
  size_t cap;
  std::list<uint64_t> l;
  std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m;
  long long hit = 0, miss = 0;
  explicit LRU(size_t c) : cap(c) { m.reserve(c * 2); }
  void touch(uint64_t a) {
    auto it = m.find(a);
    if (it != m.end()) {
      ++hit;
      l.splice(l.begin(), l, it->second);
      return;
    }
    ++miss;
    l.push_front(a);
    m[a] = l.begin();
    if (l.size() > cap) {
      m.erase(l.back());
      l.pop_back();
    }
  }
};

static int units_of(const BandGroup& G) {
  int u = 0;
  for (int w = 0; w < 4; ++w) {
    int t = 0;
    for (int h = 0; h < 2; ++h) t += (G.ra[w + 4 * h][0] >= 0) + (G.ra[w + 4 * h][1] >= 0);
    u = std::max(u, t);
  }
  return u;
}

// lists[x] = items (group, chunk) of XCD x in order; returns hit rate, prints bytes
static void simulate(const char* name, const BandPlan& p, const std::vector<std::vector<std::pair<int, int>>>& lists,
                     int M, int k_chunk, double c0) {
  const BandGeom& g = p.geom;
  long long hit = 0, miss = 0;
  double tmax = 0;
  for (int x = 0; x < 8; ++x) {
    LRU l2((4u << 20) / 128);
    struct Ev {
      double t;
      int cu;
      bool operator<(const Ev& o) const { return t > o.t; }
    };
    std::priority_queue<Ev> q;
    struct Cu {
      int item = -1, kt = 0, nk = 0;
    };
    std::vector<Cu> cus(32);
    size_t next = 0;
    const auto& L = lists[x];
    auto start = [&](int c, double t) {
      if (next >= L.size()) return;
      cus[c].item = (int)next++;
      const int ch = L[cus[c].item].second;
      const int kb = ch * k_chunk, ke = std::min(M, kb + k_chunk);
      cus[c].kt = 0;
      cus[c].nk = (ke - kb + 15) / 16;
      q.push({t, c});
    };
    for (int c = 0; c < 32; ++c) start(c, 0.0);
    while (!q.empty()) {
      Ev e = q.top();
      q.pop();
      Cu& cu = cus[e.cu];
      const BandGroup& G = p.groups[L[cu.item].first];
      const int k0 = L[cu.item].second * k_chunk + 16 * cu.kt;
      for (int i = 0; i < G.nslab; ++i) {
        const int s = G.base[i] / 64;
        for (int r = k0; r < std::min(M, k0 + 16); ++r) {
          uint64_t addr;
          if (s < g.nxs) addr = (uint64_t)r * g.kp * 4 + (uint64_t)s * 256;
          else addr = (1ull << 40) + (uint64_t)r * g.L * g.CO * 4 + (uint64_t)(s - g.nxs) * 256;
          l2.touch(addr / 128);
          l2.touch(addr / 128 + 1);
        }
      }
      const double dt = c0 + units_of(G);
      if (++cu.kt < cu.nk) q.push({e.t + dt, e.cu});
      else {
        tmax = std::max(tmax, e.t + dt);
        start(e.cu, e.t + dt);
      }
    }
    hit += l2.hit;
    miss += l2.miss;
  }
  const double in = (double)M * (g.kp + g.L * g.CO) * 4;
  std::printf("%-44s hit %5.1f %%  fabric %.2f GB (%.2fx input)  span %.0f\n", name, 100.0 * hit / (hit + miss),
              miss * 128.0 / 1e9, miss * 128.0 / in, tmax);
}

static void band_chunks_local(long long rows, int ngroups, int* nc, int* ch) {
  long long n = std::max(1, (3 * 256 + ngroups / 2) / std::max(1, ngroups));
  n = std::max(1LL, std::min(n, rows / 512 > 0 ? rows / 512 : 1));
  long long c = (rows + n - 1) / n;
  c = (c + 15) / 16 * 16;
  *ch = (int)c;
  *nc = (int)((rows + c - 1) / c);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 10240;
  const double c0 = argc > 2 ? atof(argv[2]) : 1.0;
  BandGeom g;
  band_geom(20, 20, 32, 4, 4, 2, 64, &g);
  BandPlan p;
  band_plan_build(g, &p);
  int nc, ch;
  band_chunks_local(M, (int)p.groups.size(), &nc, &ch);
  std::printf("conv2: %zu groups, %d tiles, %d chunks of %d rows\n", p.groups.size(), p.ntiles, nc, ch);
  // as built: chunk-major per XCD list
  std::vector<std::vector<std::pair<int, int>>> lists(8);
  for (int x = 0; x < 8; ++x)
    for (int c = 0; c < nc; ++c)
      for (int gi : p.xcd_groups[x]) lists[x].push_back({gi, c});
  simulate("as built (region lists, chunk-major)", p, lists, M, ch, c0);
  for (int x = 0; x < 8; ++x) {
    lists[x].clear();
    for (int gi : p.xcd_groups[x])
      for (int c = 0; c < nc; ++c) lists[x].push_back({gi, c});
  }
  simulate("region lists, group-major", p, lists, M, ch, c0);
  {
    long long distinct = 0;
    for (int x = 0; x < 8; ++x) {
      std::vector<char> seen(g.ns, 0);
      for (int gi : p.xcd_groups[x])
        for (int i = 0; i < p.groups[gi].nslab; ++i) seen[p.groups[gi].base[i] / 64] = 1;
      for (char c : seen) distinct += c;
    }
    long long staged = 0;
    for (const BandGroup& G : p.groups) staged += G.nslab;
    std::printf("slabs: %d, staged per row %lld, distinct per XCD region (sum) %lld -> floor %.2f GB\n", g.ns,
                staged, distinct, distinct * 256.0 * M / 1e9);
  }
  for (int x = 0; x < 8; ++x) {
    lists[x].clear();
    for (int c = 0; c < nc; ++c)
      for (int gi : p.xcd_groups[x]) lists[x].push_back({gi, c});
  }
  simulate("as built, equal pace (c0 = 1000)", p, lists, M, ch, 1000.0);
  // full-pace groups (4 units) of every chunk first, chunk-major; then the rest
  for (int x = 0; x < 8; ++x) {
    lists[x].clear();
    for (int pass = 0; pass < 2; ++pass)
      for (int c = 0; c < nc; ++c)
        for (int gi : p.xcd_groups[x])
          if ((units_of(p.groups[gi]) == 4) == (pass == 0)) lists[x].push_back({gi, c});
  }
  simulate("4-unit groups first, chunk-major", p, lists, M, ch, c0);
  simulate("4-unit groups first, chunk-major, c0 = 3", p, lists, M, ch, 3.0);
  for (int x = 0; x < 8; ++x) {
    lists[x].clear();
    for (int gi : p.xcd_groups[x]) lists[x].push_back({gi, 0});
  }
  simulate("one chunk (all rows per item)", p, lists, M, M, c0);
  simulate("one chunk, equal pace", p, lists, M, M, 1000.0);
  for (int ncx : {2, 6, 8, 12, 16}) {
    const int chx = ((M + ncx - 1) / ncx + 15) / 16 * 16;
    for (int x = 0; x < 8; ++x) {
      lists[x].clear();
      for (int c = 0; c < ncx; ++c)
        for (int gi : p.xcd_groups[x]) lists[x].push_back({gi, c});
    }
    char nm[64];
    std::snprintf(nm, sizeof nm, "as built, %d chunks", ncx);
    simulate(nm, p, lists, M, chx, c0);
  }
  return 0;
}
