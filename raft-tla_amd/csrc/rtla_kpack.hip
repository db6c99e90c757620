// rtla_kpack.hip -- lane-per-state row builders: the multi-shard sender's
// k_build_winners and the wave-per-state k_expand_batch (the parity seam's
// fallback for rows too wide for the level kernel).
#include "rtla_kernels_common.h"

// Sender side of the two-phase exchange: the owners
// answered every queued (fingerprint, parent) record with "new" (nonzero) or
// "seen"; the sender builds each winner ITSELF -- gathers its parent row
// (this shard's current level) into LDS, recomputes the successor's Delta,
// patches the row in place -- and appends it to ITS OWN next level with a
// local parent record.  No row crosses shards (the owner keeps only the
// fingerprint), so the next levels of the shards stay as balanced as their
// frontiers are (rtla_step re-balances what drifts).  Invariants and
// distinct coverage are evaluated here, where parent and action are known.
// LC: compiled-in layout (Layout{} = run-time Lrt), as for the level kernel.
constexpr int BW_QUEUE = 128;  // per-wave LDS queue of winner refs (u64): batches of 64 winners
__host__ __device__ constexpr int build_winners_lds_words(int W, int AW) {
  return lane_lds_words(W, AW) + 2 * BW_QUEUE;
}
template <int NS, Layout LC>
__global__ void __launch_bounds__(256)
k_build_winners(Layout Lrt, Ring cur, unsigned long long cur_base, int me,
                const unsigned long long* __restrict__ send_ref, const uint32_t* __restrict__ ans,
                const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap, Ring next,
                unsigned long long* __restrict__ parents, unsigned long long next_base, unsigned long long next_cap,
                DevCounters* ctr) {
  // A wave scans 64 records of owner p (grid.y) at a time and queues the
  // winners' refs in LDS; every 64 queued winners -- one full wave -- it
  // gathers their parent rows into LDS (one coalesced read per row), builds
  // each successor in place, reserves next-level slots with one atomic and
  // stores the rows (one coalesced write per row) and parent records.  (A
  // batch per 64 records instead would run compute_delta on the ~quarter of
  // the lanes whose record won.)
  const Layout& L = pick_layout<LC>(Lrt);
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W, AW = L.all_words;
  uint32_t* lrows = lds + wave * build_winners_lds_words(W, AW);
  const LaneWords pall{lrows + 64 * W + lane};
  unsigned long long* q = reinterpret_cast<unsigned long long*>(lrows + lane_lds_words(W, AW));
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();
  const unsigned long long p = blockIdx.y;  // owner shard
  const unsigned long long n = min(counts[p], cap);  // (reservations may run past the region: the overflow list)
  // build the first nw queued winners (q[0, nw): parent index << 16 | instance)
  auto build = [&](int nw) {
    unsigned long long obase = 0;
    if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)nw);
    obase = shfl0_u64(obase);
    if (obase + nw > next_cap && lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
    const bool act = lane < nw;
    const unsigned long long ref = act ? q[lane] : 0ull;
    const unsigned long long s = ref >> 16;  // parent: state s of the current level
    const int inst = (int)(ref & 0xffffull);
    gather_rows_lds(lrows, W, nw, [&](int r) { return ring_row(cur, readlane_u64(s, r), W); }, lane);
    wave_sync();
    uint32_t* prow = lrows + lane * W;
    if (act) {
      const FP pfp = fp_add(row_fp(prow), alllogs_delta<NS>(L, prow, pall));
      DeltaT<NS> d;
      compute_delta<NS>(L, prow, inst, d);
      const FP cfp = fp_add(pfp, delta_fp<NS>(L, prow, d));
      const int bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
      if (bad && __hip_atomic_load(&ctr->viol_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
          atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
        ctr->viol_parent = cur_base + s;
        ctr->viol_inst = inst;
        ctr->viol_in_model = 1;
        ctr->viol_child = obase + lane < next_cap ? next_base + obase + lane : ~0ull;
      }
      atomicAdd(&cov[cover_code(L, inst, d.sub)], 1u);
      materialize<NS>(L, prow, d, pall, cfp, prow);  // in place
    }
    wave_sync();
    const int nrows = obase >= next_cap ? 0 : (int)min<unsigned long long>((unsigned long long)nw, next_cap - obase);
    store_rows_ring(next, obase, nrows, W, lrows, lane);
    if (lane < nrows)
      parents[next_base + obase + lane] = (unsigned long long)me << 56 | (cur_base + s) << 16 | (unsigned long long)inst;
    wave_sync();
  };
  int qn = 0;  // winners queued (wave-uniform)
  const unsigned long long lanes_below = (1ull << lane) - 1ull;
  for (unsigned long long k0 = ((unsigned long long)blockIdx.x * wpb + wave) * 64ull; k0 < n;
       k0 += (unsigned long long)gridDim.x * wpb * 64ull) {
    const unsigned long long k = k0 + lane;
    const bool win = k < n && ans[p * cap + k] != 0u;
    const unsigned long long m = __ballot(win);
    if (win) q[qn + __popcll(m & lanes_below)] = send_ref[p * cap + k];
    qn += __popcll(m);
    wave_sync();
    if (qn >= 64) {
      build(64);
      qn -= 64;
      if (lane < qn) q[lane] = q[64 + lane];  // (the rest moves to the front: fewer than 64)
      wave_sync();
    }
  }
  if (qn) build(qn);
  __syncthreads();
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[COVER_CODES + k], (unsigned long long)cov[k]);
}

// Parity seam: every enabled successor of every input row (in-model or not),
// materialised.  out_info[k] = input index << 32 | in_model << 31 | sub << 16 | inst.
template <int NS>
__global__ void __launch_bounds__(256)
k_expand_batch(Layout L, const uint32_t* __restrict__ rows, unsigned long long n, uint32_t* __restrict__ out,
               unsigned long long* __restrict__ out_info, unsigned long long cap, DevCounters* ctr) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * wave_lds_words(W);
  uint32_t* pall = prow + even_words(W);
  FP* hsrv = reinterpret_cast<FP*>(pall + 32);
  uint32_t* stage = pall + 32 + 4 * NMAX;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wave; s < n;
       s += (unsigned long long)gridDim.x * wpb) {
    const FP pfp = load_parent<NS>(L, rows + s * (unsigned long long)W, prow, pall, hsrv, lane);
    const int nmsg = row_nmsg(L, prow);
    const int ncand = fixed + 3 * nmsg;
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      DeltaT<NS> d;
      d.enabled = 0;
      int inst = 0;
      if (q < ncand) {
        inst = candidate_inst(L, q, nmsg);
        compute_delta<NS>(L, prow, inst, d);
      }
      bool en = d.enabled != 0;
      if (en && d.err) {
        set_flag(ctr, d.err == 1 ? FLAG_SPEC_ERROR : FLAG_ROW_OVERFLOW);
        en = false;
      }
      const unsigned long long m = __ballot(en);
      const int cnt = __popcll(m);
      if (!cnt) continue;
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      unsigned long long obase = 0;
      if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)cnt);
      obase = shfl0_u64(obase);
      if (obase + cnt > cap) {
        if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
        continue;
      }
      const FP cfp = en ? fp_add(pfp, delta_fp<NS>(L, prow, d)) : FP{0, 0};
      for (int b = 0; b < cnt; b += STAGE_ROWS) {
        if (en && rank >= b && rank < b + STAGE_ROWS) materialize<NS>(L, prow, d, pall, cfp, stage + (rank - b) * W);
        wave_sync();
        const int nb = min(STAGE_ROWS, cnt - b);
        uint32_t* dst = out + (obase + b) * (unsigned long long)W;
        for (int w = lane; w < nb * W; w += 64) dst[w] = stage[w];
        wave_sync();
      }
      if (en)
        out_info[obase + rank] = s << 32 | (unsigned long long)(d.in_model ? 1u : 0u) << 31 |
                                 (unsigned long long)d.sub << 16 | (unsigned long long)inst;
    }
  }
}

namespace rtla {

template <int NS, Layout LC>
static hipError_t build_winners(const Layout& L, const Ring& cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                                const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap, const Ring& next,
                                uint64_t* parents, uint64_t next_base, uint64_t next_cap, DevCounters* ctr,
                                uint64_t max_count, hipStream_t st) {
  const size_t per = (size_t)build_winners_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  const int wpb = per * 4 <= 64 * 1024 ? 4 : (per * 2 <= 64 * 1024 ? 2 : 1);
  const size_t lds = (size_t)wpb * per;
  hipLaunchKernelGGL((k_build_winners<NS, LC>), dim3(grid_x(max_count, 1024 * wpb), nshard), dim3(64 * wpb), lds, st,
                     L, cur, (unsigned long long)cur_base, me, (const unsigned long long*)send_ref, ans,
                     (const unsigned long long*)counts, nshard, (unsigned long long)cap, next,
                     (unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)next_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_build_winners(const Layout& L, const Ring& cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                                const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap,
                                const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap,
                                DevCounters* ctr, uint64_t max_count, hipStream_t st) {
  if (!max_count) return hipSuccess;
#define RTLA_BW(LC) \
  return build_winners<LC.N, LC>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents, next_base, \
                                 next_cap, ctr, max_count, st)
  // the BASELINE layouts bench.py shards (compiled in, as for the level kernel)
  if (same_layout(L, specs::CFG2)) RTLA_BW(specs::CFG2);
  if (same_layout(L, specs::CFG1)) RTLA_BW(specs::CFG1);
  if (same_layout(L, specs::EXHAUST)) RTLA_BW(specs::EXHAUST);
  if (same_layout(L, specs::CFG3)) RTLA_BW(specs::CFG3);
  if (same_layout(L, specs::CFG4)) RTLA_BW(specs::CFG4);
#undef RTLA_BW
  switch (L.N) {
    case 1: return build_winners<1, Layout{}>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents,
                                              next_base, next_cap, ctr, max_count, st);
    case 2: return build_winners<2, Layout{}>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents,
                                              next_base, next_cap, ctr, max_count, st);
    case 3: return build_winners<3, Layout{}>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents,
                                              next_base, next_cap, ctr, max_count, st);
    case 4: return build_winners<4, Layout{}>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents,
                                              next_base, next_cap, ctr, max_count, st);
    default: return build_winners<5, Layout{}>(L, cur, cur_base, me, send_ref, ans, counts, nshard, cap, next, parents,
                                               next_base, next_cap, ctr, max_count, st);
  }
}

hipError_t launch_expand_batch(const Layout& L, const uint32_t* rows, uint64_t n, uint32_t* out, uint64_t* info,
                               uint64_t cap, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 3) / 4;
  int grid = (int)(blocks < 4096 ? blocks : 4096);
  RTLA_DISPATCH_N(L, k_expand_batch, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, rows,
                  (unsigned long long)n, out, (unsigned long long*)info, (unsigned long long)cap, ctr);
  return hipGetLastError();
}

}  // namespace rtla
