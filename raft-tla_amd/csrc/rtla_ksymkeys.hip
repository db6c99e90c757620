// rtla_ksymkeys.hip -- the SYMMETRY key kernel (one shard): orbit keys,
// seen-set probes and the new orbits' rows, for the successors the level
// kernel queued (XF_SYM_QUEUE).
//
// SYMMETRY Permutations(Server) keys the seen set by an orbit invariant
// (rtla_model.h sym_key): the least fingerprint over the images pi(s), pi in
// C(s), of each successor.  Computed inside the level kernel, the keys held
// its registers (168 VGPRs with spills at 3 waves/SIMD) and each 64-key chunk
// ran as long as its slowest lane: reachable configs[3] states compare 2.2
// images on average but the most of 64 lanes 7.5.  Here, in a kernel of its
// own, for 64 queued (parent, instance) entries per wave iteration:
//
//   1. the parents' rows are gathered into LDS and each lane turns its row
//      into the successor in place (compute_delta + materialize: the state
//      is never re-derived again);
//   2. each lane ranks its successor (sym_rank: signatures, tie groups,
//      |C(s)| images);
//   3. the wave's images -- all of them, about 2.2 x 64 -- are dealt out one
//      per lane (an exclusive scan of |C(s)| over the lanes), every lane
//      fingerprints one image of whichever successor it was dealt
//      (sym_image_fp on that successor's LDS row), and a segmented min over
//      the lanes (images of one successor are contiguous) folds them into
//      the successor's least fingerprint: the wave's time follows the total,
//      not the largest, image count;
//   4. each lane finishes its key, probes the set (load first, CAS an empty
//      slot), and the new orbits' rows -- already built, in LDS -- are
//      stored with their parent records, invariants and distinct coverage.
#include "rtla_kernels_common.h"

namespace {

constexpr int KQ = 64;  // queue entries per wave iteration (one per lane)

__device__ __forceinline__ unsigned long long shfl_u64_up(unsigned long long v, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d);
  const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d);
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

// Per-wave LDS: KQ successor rows | allLogs' words (lane-major stride 64) |
// per lane: SymRank fields, first image index, least image fingerprint.
__host__ __device__ constexpr int symkey_lds_words(int W, int AW) {
  return (KQ * W + 64 * AW + 4 * 64 + 4 * 64 + 3) & ~3;
}

}  // namespace

#ifndef RTLA_SYMKEY_WAVES_PER_EU
#define RTLA_SYMKEY_WAVES_PER_EU 2
#endif

template <int NS, Layout LC>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RTLA_SYMKEY_WAVES_PER_EU)))
k_sym_keys(Layout Lrt, Ring cur, unsigned long long cur_base, const unsigned long long* __restrict__ queue,
           const unsigned long long* __restrict__ qcount, unsigned long long qcap, Ring next,
           unsigned long long* __restrict__ parents, unsigned long long next_base, unsigned long long next_cap,
           unsigned long long* table, int tlog2, DevCounters* ctr) {
  const Layout& L = pick_layout<LC>(Lrt);
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[COVER_CODES];
  const int lane = threadIdx.x & 63;
  const int W = L.W, AW = L.all_words;
  uint32_t* rows = lds;
  const LaneWords pall{rows + KQ * W + lane};
  uint32_t* m_lo = rows + KQ * W + 64 * AW;  // [64] SymRank.lom
  uint32_t* m_cnt = m_lo + 64;               // [64] SymRank.cntm
  uint32_t* m_rad = m_cnt + 64;              // [64] SymRank.radm
  uint32_t* m_start = m_rad + 64;            // [64] first image index (exclusive scan of ncomb)
  unsigned long long* best = reinterpret_cast<unsigned long long*>(m_start + 64);  // [64][2] least image fp
  for (int k = lane; k < COVER_CODES; k += 64) cov[k] = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  const unsigned long long nq = min(*qcount, qcap);
  unsigned my_probe = 0;
  for (;;) {
    unsigned long long blk = 0;
    if (lane == 0) blk = atomicAdd(&ctr->group_next, 1ull);
    const unsigned long long k0 = shfl0_u64(blk) * KQ;
    if (k0 >= nq) break;
    const unsigned long long e = k0 + lane < nq ? queue[k0 + lane] : ~0ull;
    const bool valid = e != ~0ull;  // (~0: a hole of the level kernel's queue chunks)
    const unsigned long long s = valid ? e >> 16 : 0ull;  // parent: state s of the current level
    const int inst = valid ? (int)(e & 0xffffull) : 0;
    // 1. parents -> LDS by LDS-DMA (one global_load_lds_dword per row and
    // 64 words, every row in flight at once), then each lane turns its row
    // into its successor in place
    for (int r2 = 0; r2 < KQ; r2++) {
      const uint32_t* src = ring_row(cur, readlane_u64(s, r2), W);
      for (int c0 = 0; c0 < W; c0 += 64)
        if (c0 + lane < W)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c0 + lane),
                                           (__attribute__((address_space(3))) void*)(rows + r2 * W + c0), 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    uint32_t* const srow = rows + lane * W;
    int sub = 0;
    if (valid) {
      const FP pfp = fp_add(row_fp(srow), alllogs_delta<NS>(L, srow, pall));
      DeltaT<NS> d;
      compute_delta<NS>(L, srow, inst, d);
      sub = d.sub;
      const FP cfp = fp_add(pfp, delta_fp<NS>(L, srow, d));
      materialize<NS>(L, srow, d, pall, cfp, srow);
    }
    wave_sync();
    // 2. rank
    auto rec_at = [&](const uint32_t* row) { return [=, &L](int i, uint32_t* out) { load_rec<NS>(L, row, i, out); }; };
    auto slot_at = [&](const uint32_t* row) { return [=, &L](int q) { return slot_raw(L, row, q); }; };
    auto elec_at = [&](const uint32_t* row) { return [=, &L](int x, uint32_t* out) { elec_get(L, row, x, out); }; };
    SymRank r{0, 0, 0, 0};
    if (valid) r = sym_rank<NS>(L, rec_at(srow), row_nmsg(L, srow), slot_at(srow), row_nelec(L, srow), elec_at(srow));
    // exclusive scan of the image counts over the lanes
    int incl = r.ncomb;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const int o = __shfl_up(incl, dd);
      if (lane >= dd) incl += o;
    }
    const int total = __shfl(incl, 63);
    m_lo[lane] = r.lom;
    m_cnt[lane] = r.cntm;
    m_rad[lane] = r.radm;
    m_start[lane] = (uint32_t)(incl - r.ncomb);
    best[2 * lane] = ~0ull;
    best[2 * lane + 1] = ~0ull;
    wave_sync();
    // 3. one image per lane, in rounds of 64
    for (int b = 0; b < total; b += 64) {
      const int t = b + lane;
      const bool act = t < total;
      int j = 0;  // the successor image t belongs to: the last lane whose first image is <= t
      if (act) {
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
          if ((int)m_start[j + step] <= t) j += step;
      }
      FP f{~0ull, ~0ull};
      if (act) {
        const uint32_t* jr = rows + j * W;
        const SymRank rj{m_lo[j], m_cnt[j], m_rad[j], 0};
        f = sym_image_fp<NS>(L, rec_at(jr), row_nmsg(L, jr), slot_at(jr), row_nelec(L, jr), elec_at(jr), rj,
                             t - (int)m_start[j]);
      }
      // segmented min over the lanes (one successor's images are contiguous)
      const int seg = act ? j : -1 - lane;
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const unsigned long long oa = shfl_u64_up(f.a, dd), ob = shfl_u64_up(f.b, dd);
        const int os = __shfl_up(seg, dd);
        if (lane >= dd && os == seg && fp_less(FP{oa, ob}, f)) f = FP{oa, ob};
      }
      const int nseg = __shfl_down(seg, 1);
      if (act && (lane == 63 || nseg != seg)) {  // the segment's last lane of this round holds its min
        const FP cb{best[2 * j], best[2 * j + 1]};
        if (fp_less(f, cb)) {
          best[2 * j] = f.a;
          best[2 * j + 1] = f.b;
        }
      }
      wave_sync();
    }
    // 4. keys, probes, new orbits
    bool isnew = false;
    if (valid) {
      const FP key = fp_add(orbit_key_finish(FP{best[2 * lane], best[2 * lane + 1]}), alllogs_fp(L, srow + L.off_all));
      const unsigned long long idx = key.a >> (64 - tlog2);
      const unsigned long long seen = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      isnew = fpset_resolve_loaded(table, tlog2, key.b | 1ull, idx, seen, ctr);
      my_probe++;
    }
    const unsigned long long m = __ballot(isnew);
    if (m) {
      const int n = __popcll(m);
      unsigned long long obase = 0;
      if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)n);
      obase = shfl0_u64(obase);
      if (obase + n > next_cap && lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
      const unsigned long long child = obase + __popcll(m & below);
      const int bad = isnew ? check_invariants<NS>(L, srow, (const DeltaT<NS>*)nullptr) : 0;
      if (claim_violation(ctr, bad, lane)) {
        ctr->viol_parent = cur_base + s;
        ctr->viol_inst = inst;
        ctr->viol_in_model = 1;
        ctr->viol_child = child < next_cap ? next_base + child : ~0ull;
      }
      {  // distinct coverage, aggregated over equal codes
        const int code = isnew ? cover_code(L, inst, sub) : -1;
        const int c0 = __shfl(code, __builtin_ctzll(m));
        const bool same = isnew && code == c0;
        const int n0 = __popcll(__ballot(same));
        if (lane == 0) atomicAdd(&cov[c0], (unsigned)n0);
        if (isnew && !same) atomicAdd(&cov[code], 1u);
      }
      // the rows, already built: one coalesced store per new orbit
      unsigned long long mm = m;
      for (int r2 = 0; mm; r2++) {
        const int l = __builtin_ctzll(mm);
        mm &= mm - 1;
        if (obase + r2 < next_cap) {
          uint32_t* dst = ring_row(next, obase + r2, W);
          for (int w = lane; w < W; w += 64) dst[w] = rows[l * W + w];
        }
      }
      if (isnew && child < next_cap) parents[next_base + child] = (cur_base + s) << 16 | (unsigned long long)inst;
    }
    wave_sync();  // (the LDS rows are refilled next)
  }
  for (int off = 32; off > 0; off >>= 1) my_probe += __shfl_down(my_probe, off);
  if (lane == 0 && my_probe) atomicAdd(&ctr->probes, (unsigned long long)my_probe);
  wave_sync();
  for (int k = lane; k < COVER_CODES; k += 64)
    if (cov[k]) atomicAdd(&ctr->cover[COVER_CODES + k], (unsigned long long)cov[k]);
}

namespace rtla {

template <int NS, Layout LC>
static hipError_t sym_keys(const Layout& L, const Ring& cur, uint64_t cur_base, const uint64_t* queue,
                           const uint64_t* qcount, uint64_t qcap, const Ring& next, uint64_t* parents,
                           uint64_t next_base, uint64_t next_cap, uint64_t* table, int tlog2, DevCounters* ctr,
                           hipStream_t st) {
  auto kfn = k_sym_keys<NS, LC>;
  const size_t lds = (size_t)symkey_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  static int per_cu = 0;  // persistent one-wave blocks: the resident capacity
  if (!per_cu && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 64, lds) != hipSuccess || per_cu < 1))
    per_cu = 4;
  hipError_t e = hipMemsetAsync(&ctr->group_next, 0, sizeof(ctr->group_next), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kfn, dim3((unsigned)(device_cus() * per_cu)), dim3(64), lds, st, L, cur,
                     (unsigned long long)cur_base, (const unsigned long long*)queue,
                     (const unsigned long long*)qcount, (unsigned long long)qcap, next, (unsigned long long*)parents,
                     (unsigned long long)next_base, (unsigned long long)next_cap, (unsigned long long*)table, tlog2,
                     ctr);
  return hipGetLastError();
}

bool launch_sym_keys_supported(const Layout& L) {
  return (size_t)symkey_lds_words(L.W, L.all_words) * sizeof(uint32_t) <= 64 * 1024;
}

hipError_t launch_sym_keys(const Layout& L, const Ring& cur, uint64_t cur_base, const uint64_t* queue,
                           const uint64_t* qcount, uint64_t qcap, const Ring& next, uint64_t* parents,
                           uint64_t next_base, uint64_t next_cap, uint64_t* table, int tlog2, DevCounters* ctr,
                           hipStream_t st) {
  if ((size_t)symkey_lds_words(L.W, L.all_words) * sizeof(uint32_t) > 64 * 1024) return hipErrorNotSupported;
  if (same_layout(L, specs::CFG4))
    return sym_keys<specs::CFG4.N, specs::CFG4>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base,
                                                next_cap, table, tlog2, ctr, st);
  switch (L.N) {
    case 1: return sym_keys<1, Layout{}>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base, next_cap,
                                         table, tlog2, ctr, st);
    case 2: return sym_keys<2, Layout{}>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base, next_cap,
                                         table, tlog2, ctr, st);
    case 3: return sym_keys<3, Layout{}>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base, next_cap,
                                         table, tlog2, ctr, st);
    case 4: return sym_keys<4, Layout{}>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base, next_cap,
                                         table, tlog2, ctr, st);
    default: return sym_keys<5, Layout{}>(L, cur, cur_base, queue, qcount, qcap, next, parents, next_base, next_cap,
                                          table, tlog2, ctr, st);
  }
}

}  // namespace rtla
