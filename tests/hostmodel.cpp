// hostmodel.cpp -- TEST INFRASTRUCTURE: the product's model code
// (raft-tla_amd/csrc/rtla_model.h, written once for host and device)
// compiled for the host, so the CPU test suite can check the semantics the
// kernels evaluate -- successor generation, incremental fingerprints, row
// building -- against the oracles without a GPU.  The product never runs
// this: its only expansion path is the HIP level kernel (librtla.so).
//
// hm_expand mirrors the level kernel's per-successor work: compute_delta on
// the parent row, the fingerprint derived incrementally (parent fp +
// allLogs' change + delta_fp), the child row materialised from the patches.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "rtla_model.h"

using namespace rtla;

extern "C" {

// layout of a model (K, E: bag slots, election records); 0 on success
int hm_layout(int n, int v, int t, int l, int c, int m, int k, int e, int inv, int sym, int* words) {
  Layout L;
  if (make_layout(&L, n, v, t, l, c, m, k, e, inv) != 0) return -1;
  *words = L.W;
  (void)sym;
  return 0;
}

// Every enabled successor of each input row: out rows, info[k] = input index
// << 32 | in_model << 31 | sub << 16 | instance.  Returns the count, or -1 if
// cap is too small, -2 on a row-capacity error, -3 on a spec error.
long hm_expand(int n, int v, int t, int l, int c, int m, int k, int e, int inv, const uint32_t* rows, size_t nrows,
               uint32_t* out, uint64_t* info, size_t cap) {
  Layout L;
  if (make_layout(&L, n, v, t, l, c, m, k, e, inv) != 0) return -4;
  const int W = L.W;
  size_t cnt = 0;
  std::vector<uint32_t> pall(L.all_words + 1);
  for (size_t s = 0; s < nrows; s++) {
    const uint32_t* row = rows + s * W;
    const FP pfp = fp_add(row_fp(row), alllogs_delta<0>(L, row, pall.data()));
    for (int inst = 0; inst < L.fam[F_COUNT]; inst++) {
      Delta d;
      compute_delta<0>(L, row, inst, d);
      if (!d.enabled) continue;
      if (d.err) return d.err == 1 ? -3 : -2;
      if (cnt >= cap) return -1;
      const FP cfp = fp_add(pfp, delta_fp<0>(L, row, d));
      materialize<0>(L, row, d, pall.data(), cfp, out + cnt * W);
      info[cnt] = (uint64_t)s << 32 | (uint64_t)(d.in_model ? 1u : 0u) << 31 | (uint64_t)d.sub << 16 | (uint64_t)inst;
      cnt++;
    }
  }
  return (long)cnt;
}

// Fingerprint of a row from scratch.
int hm_fingerprint(int n, int v, int t, int l, int c, int m, int k, int e, int inv, const uint32_t* row, uint64_t* out) {
  Layout L;
  if (make_layout(&L, n, v, t, l, c, m, k, e, inv) != 0) return -4;
  const FP f = row_fingerprint(L, row);
  out[0] = f.a;
  out[1] = f.b;
  return 0;
}

}  // extern "C"
