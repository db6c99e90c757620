// symstat -- orbit-key workload statistics over sampled configs[3] successors
// (tools/sym_dump.py writes them): how many permutation images the key
// computes per successor (sym_rank's |C(s)|), how many of those images are
// distinct (the rest are automorphisms a better twin test would skip), what
// the slowest lane of a 64-successor chunk computes, and the same for a
// refined signature (one round of neighbour refinement).  Diagnostic only.
//
//   hipcc -O2 -std=c++20 -I raft-tla_amd/csrc tools/symstat.cpp -o /tmp/symstat
//   /tmp/symstat gpurun_out/symdump
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "rtla_model.h"

using namespace rtla;

static std::vector<uint32_t> load_npy_u32(const std::string& path, size_t* rows, size_t* cols, int words = 1) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) { perror(path.c_str()); exit(1); }
  char magic[10];
  if (fread(magic, 1, 10, f) != 10) exit(1);
  const unsigned hl = (unsigned char)magic[8] | (unsigned char)magic[9] << 8;
  std::string h(hl, ' ');
  if (fread(&h[0], 1, hl, f) != hl) exit(1);
  size_t a = h.find("'shape': (");
  *rows = strtoull(h.c_str() + a + 10, nullptr, 10);
  size_t comma = h.find(',', a + 10);
  *cols = strtoull(h.c_str() + comma + 1, nullptr, 10);
  std::vector<uint32_t> v(*rows * *cols * words);
  if (fread(v.data(), 4, v.size(), f) != v.size()) exit(1);
  fclose(f);
  return v;
}

// Refined signatures: sig1_i folds in, as order-free sums, the round-0
// signatures of the servers i's messages and record name (equivariant: a
// server's name never enters, only the signature of the server it names).
template <int NS>
static SymRank sym_rank_refined(const Layout& L, const uint32_t* row) {
  constexpr int SW = 3 + NS;
  auto rec_of = [&](int i, uint32_t* out) { load_rec<NS>(L, row, i, out); };
  const int nmsg = row_nmsg(L, row);
  auto slot_of = [&](int q) { return slot_raw(L, row, q); };
  uint32_t ms[NS] = {}, mr[NS] = {};
  const uint64_t sm = (1ull << L.b_sid) - 1ull;
  for (int q = 0; q < nmsg; q++) {
    const uint64_t v = slot_of(q);
    if (!v) continue;
    const uint32_t src = (uint32_t)(v >> 2 & sm), dst = (uint32_t)(v >> (2 + L.b_sid) & sm);
    const uint64_t anon = v & ~(sm << 2 | sm << (2 + L.b_sid));
    const uint32_t c = mix32((uint32_t)anon ^ mix32((uint32_t)(anon >> 32) + 0x632be5abu));
    ms[src] += c;
    mr[dst] += mix32(c ^ 0x5bd1e995u);
  }
  uint64_t sig[NS];
  for (int i = 0; i < NS; i++) {
    uint32_t rec[SW];
    rec_of(i, rec);
    sig[i] = (uint64_t)srv_sig<NS>(i, rec) << 32 | mix32(ms[i] ^ mix32(mr[i] + 0x27d4eb2fu));
  }
  // round 1
  uint32_t s0[NS];
  for (int i = 0; i < NS; i++) s0[i] = mix32((uint32_t)sig[i] ^ (uint32_t)(sig[i] >> 32));
  uint32_t add[NS] = {};
  for (int q = 0; q < nmsg; q++) {
    const uint64_t v = slot_of(q);
    if (!v) continue;
    const uint32_t src = (uint32_t)(v >> 2 & sm), dst = (uint32_t)(v >> (2 + L.b_sid) & sm);
    const uint64_t anon = v & ~(sm << 2 | sm << (2 + L.b_sid));
    const uint32_t c = mix32((uint32_t)anon ^ mix32((uint32_t)(anon >> 32) + 0x1b873593u));
    add[src] += mix32(c ^ s0[dst]);
    add[dst] += mix32(c ^ s0[src] ^ 0x9e3779b9u);
  }
  for (int i = 0; i < NS; i++) {
    uint32_t rec[SW];
    rec_of(i, rec);
    const uint32_t w0 = rec[0], nm = rec[2];
    for (int j = 0; j < NS; j++) {
      if (j == i) continue;
      const uint32_t t = (s_vresp(w0) >> j & 1u) | (s_vgrant(w0) >> j & 1u) << 1 | (s_vlp(w0) >> j & 1u) << 2 |
                         (s_voted(w0) == (uint32_t)j ? 8u : 0u) | nm_next(nm, j) << 4 | nm_match(nm, j) << 8;
      add[i] += mix32(mix32(t ^ mix32(rec[3 + j] + 0x85ebca6bu)) ^ s0[j]);
    }
  }
  const int nelec = row_nelec(L, row);
  for (int e = 0; e < nelec; e++) {
    uint32_t er[2 + NS];
    elec_get(L, row, e, er);
    const uint32_t w0 = er[0];
    const uint32_t ld = (w0 >> 4) & 7u, votes = (w0 >> 7) & 31u, dom = (w0 >> 12) & 31u;
    const uint32_t ebase = mix32((w0 & 15u) ^ mix32(er[1] + 0xc2b2ae35u));
    for (int i = 0; i < NS; i++) {
      const uint32_t t = (ld == (uint32_t)i ? 1u : 0u) | (votes >> i & 1u) << 1 | (dom >> i & 1u) << 2;
      if (t) add[i] += mix32(ebase ^ mix32(t ^ mix32(er[2 + i] + 0x27d4eb2fu)));
    }
  }
  for (int i = 0; i < NS; i++) sig[i] = (sig[i] & ~0xffffffffull) | mix32((uint32_t)sig[i] ^ mix32(add[i]));
  SymRank r{0, 0, 0, 1};
  for (int i = 0; i < NS; i++) {
    int l = 0, c = 0, b = 0;
    for (int j = 0; j < NS; j++) {
      l += sig[j] < sig[i] ? 1 : 0;
      c += sig[j] == sig[i] ? 1 : 0;
      if (j < i) b += sig[j] == sig[i] ? 1 : 0;
    }
    r.lom |= (uint32_t)l << (3 * i);
    r.cntm |= (uint32_t)c << (3 * i);
    r.radm |= (uint32_t)(c - b) << (3 * i);
    r.ncomb *= c - b;
  }
  return r;
}

template <int NS>
static int distinct_images(const Layout& L, const uint32_t* row, const SymRank& r) {
  auto rec_of = [&](int i, uint32_t* out) { load_rec<NS>(L, row, i, out); };
  auto slot_of = [&](int q) { return slot_raw(L, row, q); };
  auto elec_of = [&](int e, uint32_t* out) { elec_get(L, row, e, out); };
  std::set<std::pair<uint64_t, uint64_t>> s;
  for (int k = 0; k < r.ncomb; k++) {
    const FP f = sym_image_fp<NS>(L, rec_of, row_nmsg(L, row), slot_of, row_nelec(L, row), elec_of, r, k);
    s.insert({f.a, f.b});
  }
  return (int)s.size();
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "gpurun_out/symdump";
  size_t n = 0, w = 0, ni = 0, wi = 0;
  std::vector<uint32_t> rows = load_npy_u32(dir + "/succ.npy", &n, &w);
  // succ_info.npy is int64 (parent, inst, sub): read as u32 pairs
  std::vector<uint32_t> info = load_npy_u32(dir + "/succ_info.npy", &ni, &wi, 2);
  Layout L = layout_of(5, 1, 3, 2, 1, 0, 20, 10, 0);
  L.sym = 1;
  if ((size_t)L.W != w) {
    fprintf(stderr, "row width %zu, layout %d\n", w, L.W);
    return 1;
  }
  std::vector<int> cur(n), twin2(n), ref(n), dist(n);
  std::map<int, long> hc, hr, hd;
  long sc = 0, sr = 0, sd = 0;
  for (size_t k = 0; k < n; k++) {
    const uint32_t* row = rows.data() + k * w;
    int perms = 0;
    (void)orbit_key_row<5>(L, row, &perms);
    cur[k] = perms;
    const SymRank rr = sym_rank_refined<5>(L, row);
    ref[k] = rr.ncomb;
    // distinct images among the current C(s) (after sym_rank's twin pruning)
    auto rec_of = [&](int i, uint32_t* out) { load_rec<5>(L, row, i, out); };
    auto slot_of = [&](int q) { return slot_raw(L, row, q); };
    auto elec_of = [&](int e, uint32_t* out) { elec_get(L, row, e, out); };
    const SymRank r0 = sym_rank<5>(L, rec_of, row_nmsg(L, row), slot_of, row_nelec(L, row), elec_of);
    dist[k] = distinct_images<5>(L, row, r0);
    hc[cur[k]]++; hr[ref[k]]++; hd[dist[k]]++;
    sc += cur[k]; sr += ref[k]; sd += dist[k];
  }
  auto show = [&](const char* name, std::map<int, long>& h, long s) {
    printf("%-28s mean %.3f  hist:", name, (double)s / n);
    for (auto& [k, v] : h) printf(" %d:%ld", k, v);
    printf("\n");
  };
  printf("%zu successors\n", n);
  show("images, current signature", hc, sc);
  show("distinct images", hd, sd);
  show("images, refined signature", hr, sr);
  // chunks: per 32 consecutive parents, successors instance-major, 64 at a time
  auto chunk_max = [&](const std::vector<int>& v) {
    std::vector<std::pair<std::pair<long, long>, int>> order;  // ((group, inst), parent) -> value
    double tot = 0;
    long chunks = 0;
    std::map<long, std::vector<std::pair<std::pair<long, long>, int>>> by_group;
    for (size_t k = 0; k < n; k++) {
      const long parent = info[2 * (k * wi)], inst = info[2 * (k * wi + 1)];
      by_group[parent / 32].push_back({{inst, parent}, v[k]});
    }
    for (auto& [g, vec] : by_group) {
      std::sort(vec.begin(), vec.end(), [](auto& a, auto& b) { return a.first < b.first; });
      for (size_t b = 0; b < vec.size(); b += 64) {
        int m = 0;
        for (size_t j = b; j < std::min(vec.size(), b + 64); j++) m = std::max(m, vec[j].second);
        tot += m;
        chunks++;
      }
    }
    return tot / std::max(1l, chunks);
  };
  printf("slowest lane per 64-chunk: current %.3f  distinct %.3f  refined %.3f\n", chunk_max(cur), chunk_max(dist),
         chunk_max(ref));
  return 0;
}
