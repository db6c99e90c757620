// rtla_kernels.hip -- gfx950 kernels of the BFS hot path.
//
// One BFS level = one launch of k_expand over the current frontier:
//   * one wavefront per frontier state: the 64 lanes copy the packed row into
//     LDS (coalesced); lanes 0..N-1 hash the parent's server records and lane
//     N derives the per-parent allLogs' (raft.tla:465), all into LDS;
//   * each lane evaluates one action instance of Next (raft.tla:454-463) as a
//     Delta against the LDS row (rtla_model.h): every lane reads the same
//     parent words (LDS broadcast, no bank conflicts) and the Delta stays in
//     VGPRs (the model is instantiated per server count, NS);
//   * the successor's 128-bit fingerprint is the parent's plus the Delta's
//     component change (no full re-hash);
//   * in-model successors probe the open-addressing fingerprint set in HBM
//     with one 8-byte CAS per probe (home slot from fp.a, key fp.b | 1):
//     one memory round trip whether the state is new or seen;
//   * new successors are compacted by ballot + popcount prefix, built in a
//     16-row LDS staging tile and written to the next frontier as contiguous,
//     coalesced ranges;
//   * invariants are checked on every new and every out-of-model successor.
#include "rtla_kernels_common.h"

using namespace rtla;

template <int NS>
__global__ void __launch_bounds__(256)
k_expand(Layout L, Ring cur, unsigned long long s_begin, unsigned long long s_end,
         unsigned long long cur_base, Ring next, unsigned long long* __restrict__ parents,
         unsigned long long next_base, unsigned long long next_cap, unsigned long long* table, int tlog2,
         DevCounters* ctr, ShardBox box) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[2 * COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * wave_lds_words(W);
  uint32_t* pall = prow + even_words(W);
  FP* hsrv = reinterpret_cast<FP*>(pall + 32);
  uint32_t* stage = pall + 32 + 4 * NMAX;
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();

  unsigned long long my_gen = 0, my_probe = 0;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = s_begin + (unsigned long long)blockIdx.x * wpb + wave; s < s_end;
       s += (unsigned long long)gridDim.x * wpb) {
    const FP pfp = load_parent<NS>(L, ring_row(cur, s, W), prow, pall, hsrv, lane);
    // SYMMETRY: allLogs' is the same for every successor (raft.tla:465)
    const FP afp = L.sym ? alllogs_fp(L, pall) : FP{0, 0};
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
      my_gen += en ? 1 : 0;
      bool isnew = false;
      FP cfp{0, 0};
      if (en && d.in_model) {
        cfp = fp_add(pfp, delta_fp<NS>(L, prow, d, d.srv >= 0 ? &hsrv[d.srv] : nullptr));
        // seen-set key: the state's own fingerprint, or under SYMMETRY its
        // orbit key (least fingerprint over the server permutations)
        const FP key = L.sym ? successor_orbit_key<NS>(L, prow, d, afp) : cfp;
        const int owner = fp_owner(key, box.nshard);
        if (owner == box.me) {
          my_probe++;
          int r = fpset_insert(table, tlog2, key);
          if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
          isnew = r == 1;
        } else {
          // Another shard owns this fingerprint: queue (fp, parent, instance);
          // the owner answers new/seen and this shard ships it the winner.
          unsigned long long slot = atomicAdd(&box.out_count[owner], 1ull);
          if (slot < box.cap) {
            unsigned long long k = (unsigned long long)owner * box.cap + slot;
            box.send_fp[2 * k] = key.a;
            box.send_fp[2 * k + 1] = key.b;
            box.send_ref[k] = s << 16 | (unsigned long long)inst;
          } else {
            set_flag(ctr, FLAG_OUTBOX_FULL);
          }
        }
      }
      if (en) {
        int code = cover_code(L, inst, d.sub);
        atomicAdd(&cov[code], 1u);
        if (isnew) atomicAdd(&cov[COVER_CODES + code], 1u);
      }
      const unsigned long long m = __ballot(isnew);
      const int cnt = __popcll(m);
      unsigned long long obase = 0;
      int rank = 0;
      if (cnt) {
        rank = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)cnt);
        obase = shfl0_u64(obase);
        if (obase + cnt > next_cap) {
          if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
        } else {
          // stage and write out STAGE_ROWS new rows at a time
          for (int b = 0; b < cnt; b += STAGE_ROWS) {
            if (isnew && rank >= b && rank < b + STAGE_ROWS)
              materialize<NS>(L, prow, d, pall, cfp, stage + (rank - b) * W);
            wave_sync();
            store_rows_ring(next, obase + b, min(STAGE_ROWS, cnt - b), W, stage, lane);
            wave_sync();
          }
          if (isnew)
            parents[next_base + obase + rank] =
                (unsigned long long)box.me << 56 | (cur_base + s) << 16 | (unsigned long long)inst;
        }
      }
      if (en && (isnew || !d.in_model)) {
        int bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
        if (bad && __hip_atomic_load(&ctr->viol_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
          ctr->viol_parent = cur_base + s;
          ctr->viol_inst = inst;
          ctr->viol_in_model = d.in_model;
          ctr->viol_child = isnew ? next_base + obase + rank : ~0ull;
        }
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    my_gen += __shfl_down(my_gen, off);
    my_probe += __shfl_down(my_probe, off);
  }
  if (lane == 0 && my_gen) atomicAdd(&ctr->generated, my_gen);
  if (lane == 0 && my_probe) atomicAdd(&ctr->probes, my_probe);
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[k], (unsigned long long)cov[k]);
}
// Owner side of the exchange: insert the fingerprints other shards sent and
// answer each record with 0 (seen) or 1 + its dense rank among the new
// fingerprints from that source (the sender uses the rank as the row slot it
// ships the materialised state into).  Region p holds counts[p] records.
__global__ void k_insert_remote(const unsigned long long* __restrict__ recv_fp,
                                const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap,
                                unsigned long long* table, int tlog2, uint32_t* __restrict__ ans,
                                unsigned long long* __restrict__ new_count, DevCounters* ctr) {
  // grid.y = source shard p; lanes of a wave share p, so one atomic per wave
  // hands out the dense ranks of its new fingerprints
  const unsigned long long p = blockIdx.y;
  const unsigned long long n = counts[p];
  const int lane = threadIdx.x & 63;
  unsigned probes = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long k0 = (unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); k0 < n;
       k0 += stride) {
    const unsigned long long k = k0 + lane;
    int r = 0;
    if (k < n) {
      const unsigned long long i = p * cap + k;
      const FP f{recv_fp[2 * i], recv_fp[2 * i + 1]};
      if (f.a | f.b) {  // 0:0 = a hole in the sender's outbox chunk
        r = fpset_insert(table, tlog2, f);
        if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
        probes++;
      }
    }
    const unsigned long long m = __ballot(r == 1);
    unsigned long long b = 0;
    if (m) {
      if (lane == 0) b = atomicAdd(&new_count[p], (unsigned long long)__popcll(m));
      b = shfl0_u64(b);
    }
    if (k < n) ans[p * cap + k] = r == 1 ? (uint32_t)(b + __popcll(m & ((1ull << lane) - 1ull))) + 1u : 0u;
  }
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off);
  if (lane == 0 && probes) atomicAdd(&ctr->probes, (unsigned long long)probes);
}

// Sender side: materialise the queued successors whose owner answered "new"
// with a rank in [lo, hi) into the owner's row region (row + parent record,
// RW = W + 2 words per slot).  Invariants are checked here, where parent and
// action are known; a violation is recorded against the local parent.
template <int NS>
__global__ void __launch_bounds__(256)
k_pack_rows(Layout L, Ring cur, unsigned long long cur_base, int me,
            const unsigned long long* __restrict__ send_ref, const uint32_t* __restrict__ ans,
            const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap, unsigned long long lo,
            unsigned long long hi, uint32_t* __restrict__ rows, unsigned long long rows_cap, DevCounters* ctr) {
  // A wave scans 64 records of owner p (grid.y), compacts the winners of
  // this sub-round, gathers their parent rows into LDS (one coalesced read
  // per row), builds each successor in place and ships row + parent record
  // to the slot the owner's answer names (one coalesced write per row).
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W, AW = L.all_words, RW = W + 2;
  uint32_t* lrows = lds + wave * lane_lds_words(W, AW);
  const LaneWords pall{lrows + 64 * W + lane};
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();
  const unsigned long long p = blockIdx.y;  // owner shard
  const unsigned long long n = counts[p];
  const unsigned long long below = (1ull << lane) - 1ull;
  for (unsigned long long k0 = ((unsigned long long)blockIdx.x * wpb + wave) * 64ull; k0 < n;
       k0 += (unsigned long long)gridDim.x * wpb * 64ull) {
    const unsigned long long k = k0 + lane;
    const unsigned long long i = p * cap + k;
    const unsigned long long a = k < n ? ans[i] : 0ull;
    const bool win = a != 0 && a - 1 >= lo && a - 1 < hi;
    const unsigned long long m = __ballot(win);
    if (!m) continue;
    const int nw = __popcll(m);
    // compact: winner number r of this wave = lane w_r
    int r_of_lane = __popcll(m & below);
    unsigned long long ref = win ? send_ref[i] : 0ull;
    unsigned long long dslot = win ? a - 1 - lo : 0ull;
    // lane r takes the r-th winner's (ref, dslot)
    int src_lane = 0;
    {
      unsigned long long mm = m;
      for (int r = 0; r < nw; r++) {
        const int l = __builtin_ctzll(mm);
        mm &= mm - 1;
        if (lane == r) src_lane = l;
      }
    }
    (void)r_of_lane;
    ref = shfl_u64(ref, src_lane);
    dslot = shfl_u64(dslot, src_lane);
    const bool act = lane < nw;
    const unsigned long long s = ref >> 16;
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
        ctr->viol_child = ~0ull;
      }
      atomicAdd(&cov[cover_code(L, inst, d.sub)], 1u);
      materialize<NS>(L, prow, d, pall, cfp, prow);  // in place
    }
    wave_sync();
    for (int r = 0; r < nw; r++) {
      const unsigned long long ds = readlane_u64(dslot, r);
      uint32_t* dst = rows + (p * rows_cap + ds) * (unsigned long long)RW;
      for (int w = lane; w < W; w += 64) dst[w] = lrows[r * W + w];
      if (lane == 0) {
        const unsigned long long pr =
            (unsigned long long)me << 56 | (cur_base + readlane_u64(s, r)) << 16 | (unsigned long long)__builtin_amdgcn_readlane(inst, r);
        dst[W] = (uint32_t)pr;
        dst[W + 1] = (uint32_t)(pr >> 32);
      }
    }
    wave_sync();
  }
  __syncthreads();
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[COVER_CODES + k], (unsigned long long)cov[k]);
}

// Owner side: append the received rows to the next frontier (one wave per
// row, coalesced copy) with their cross-shard parent records.
__global__ void k_unpack_rows(int W, const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ counts,
                              const unsigned long long* __restrict__ bases, int nshard, unsigned long long rows_cap,
                              Ring next, unsigned long long* __restrict__ parents,
                              unsigned long long next_base, unsigned long long next_cap, DevCounters* ctr) {
  // grid.y = source shard p; its rows land at the contiguous slots bases[p] + k
  // (bases from k_part_counts: no per-row atomics)
  const unsigned long long p = blockIdx.y;
  const unsigned long long n = counts[p], base = bases[p];
  const int lane = threadIdx.x & 63;
  const int RW = W + 2;
  const unsigned long long wv = (blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x) >> 6;
  const unsigned long long nw = ((unsigned long long)gridDim.x * blockDim.x) >> 6;
  for (unsigned long long k = wv; k < n; k += nw) {
    const unsigned long long o = base + k;
    if (o >= next_cap) {
      if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
      continue;
    }
    const uint32_t* src = rows + (p * rows_cap + k) * (unsigned long long)RW;
    uint32_t* dst = ring_row(next, o, W);
    for (int w = lane; w < W; w += 64) dst[w] = src[w];
    if (lane == 0) parents[next_base + o] = (unsigned long long)src[W] | (unsigned long long)src[W + 1] << 32;
  }
}

// rows_in[p] = the part [lo, lo + rc) of the new_count[p] rows owner-side.
// and bases[p] = the next-frontier slot of its first row; advances next_count.
__global__ void k_part_counts(const unsigned long long* __restrict__ new_count, int nshard, unsigned long long lo,
                              unsigned long long rc, unsigned long long* __restrict__ rows_in,
                              unsigned long long* __restrict__ bases, DevCounters* ctr) {
  if (threadIdx.x != 0) return;
  unsigned long long b = ctr->next_count;
  for (int p = 0; p < nshard; p++) {
    const unsigned long long n = new_count[p];
    const unsigned long long r = n > lo ? min(n - lo, rc) : 0ull;
    rows_in[p] = r;
    bases[p] = b;
    b += r;
  }
  ctr->next_count = b;
}

// Insert the fingerprints of `n` rows (Init).  new_flags[i] = 1 if new.
__global__ void k_insert_rows(Layout L, const uint32_t* rows, unsigned long long n, unsigned long long* table,
                              int tlog2, int* new_flags, DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  FP f = row_fp(rows + i * (unsigned long long)L.W);
  int r = fpset_insert(table, tlog2, f);
  if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
  new_flags[i] = r == 1;
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

// Synthetic microbench input (BASELINE configs[4], rtla_synth.h): input states
// first .. first + n - 1 as rows 0 .. n - 1 of `out`.  One lane builds one
// row in LDS; the wave stores its 64 rows with coalesced stores.
__global__ void __launch_bounds__(64)
k_random_rows(Layout L, unsigned long long seed, unsigned long long first, unsigned long long n,
              unsigned long long pool, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int W = L.W;
  for (unsigned long long g = (unsigned long long)blockIdx.x * 64; g < n; g += (unsigned long long)gridDim.x * 64) {
    const int nv = (int)min<unsigned long long>(64ull, n - g);
    if (lane < nv) random_state(L, seed, synth_state_id(seed, first + g + lane, pool), lds + lane * W);
    wave_sync();
    uint32_t* dst = out + g * (unsigned long long)W;
    for (int w = lane; w < nv * W; w += 64) dst[w] = lds[w];
    wave_sync();
  }
}

// Microbenchmark kernel: random 8-B CAS inserts into a table (calibrates the
// random-access roofline of the fingerprint set).
__global__ void k_probe_bench(unsigned long long* table, int tlog2, unsigned long long n, unsigned long long seed,
                              DevCounters* ctr, int load_first) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long got = 0;
  for (; i < n; i += stride) {
    FP f = hash_u64(seed, i);
    if (load_first) {
      const unsigned long long idx = f.a >> (64 - tlog2);
      const unsigned long long v = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      got += fpset_resolve_loaded(table, tlog2, f.b | 1ull, idx, v, ctr) ? 1 : 0;
    } else {
      got += fpset_insert(table, tlog2, f) == 1;
    }
  }
  for (int off = 32; off > 0; off >>= 1) got += __shfl_down(got, off);
  if ((threadIdx.x & 63) == 0 && got) atomicAdd(&ctr->next_count, got);
}

// ---------------------------------------------------------------- launch ----
namespace rtla {

size_t expand_lds_bytes(const Layout& L, int wpb) {
  return (size_t)wpb * (size_t)wave_lds_words(L.W) * sizeof(uint32_t);
}

int expand_lane_wpb(const Layout& L) {
  const size_t per = (size_t)lane_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  if (per > 64 * 1024) return 0;
  return per * 4 <= 64 * 1024 ? 4 : (per * 2 <= 64 * 1024 ? 2 : 1);
}


int expand_compact_wpb(const Layout& L) {
  const size_t per = (size_t)compact_lds_words(L.W, L.all_words, compact_group(L), L.sym, true) * sizeof(uint32_t);
  // one wave may use up to the CU's 160 KiB of LDS; instance ids fit 8 bits per 64-instance window
  if (per > 160 * 1024 || ((L.fam[F_COUNT] + 63) / 64) * 64 > 256) return 0;
  return per * 4 <= 64 * 1024 ? 4 : (per * 2 <= 64 * 1024 ? 2 : 1);
}

int expand_blocks_per_cu(const Layout& L) {
  size_t per = expand_lds_bytes(L, 4) + 2 * COVER_CODES * sizeof(unsigned int);
  int b = (int)((160u * 1024u) / per);
  return b < 1 ? 1 : (b > 8 ? 8 : b);
}

#define RTLA_DISPATCH_N(L, KERNEL, ...)                        \
  switch ((L).N) {                                             \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break; \
  }

hipError_t launch_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end, uint64_t cur_base,
                         const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap, uint64_t* table,
                         int tlog2, DevCounters* ctr, const ShardBox& box, int grid, hipStream_t st, int xflags,
                         uint64_t* sent, hipEvent_t mid) {
  if (s_end <= s_begin) return hipSuccess;
  const int cwpb = expand_compact_wpb(L);
  if (cwpb > 0 && !(xflags & XF_WAVE_KERNEL) && (box.nshard == 1 || sent)) {
    const CompactArgs a{L,         box.nshard > 1, cur,      s_begin, s_end,  cur_base, next,   parents, next_base,
                        next_cap,  table,          tlog2,    ctr,     box,    st,       xflags, sent,
                        (xflags & XF_BLOCK4) ? cwpb : 1};  // one-wave workgroups by default
    hipError_t e = hipSuccess;
    bool done = false;
    // the compiled-in BASELINE layouts first, then the run-time layout
    if (!(xflags & XF_NO_SPECIAL)) {
      e = launch_compact_spec_a(a, &done);
      if (!done) e = launch_compact_spec_b(a, &done);
    }
#ifndef RTLA_EXP_MINIMAL  // perf experiments: compiled-in layouts only (fast builds)
    if (!done && L.sym) e = launch_compact_sym(a, &done);
    if (!done) e = launch_compact_generic_a(a, &done);
    if (!done) e = launch_compact_generic_b(a, &done);
#endif
    if (!done) return hipErrorNotSupported;
    if (e != hipSuccess) return e;
    if (mid) {
      e = hipEventRecord(mid, st);
      if (e != hipSuccess) return e;
    }
    return hipGetLastError();
  }
  // one wave per state: rows too wide for the compacting kernel's LDS tile
  // (or forced, XF_WAVE_KERNEL)
  RTLA_DISPATCH_N(L, k_expand, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, cur,
                  (unsigned long long)s_begin, (unsigned long long)s_end, (unsigned long long)cur_base, next,
                  (unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)next_cap,
                  (unsigned long long*)table, tlog2, ctr, box);
  return hipGetLastError();
}

static unsigned grid_x(uint64_t n, int per_block) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per_block - 1) / per_block, 4096));
}

hipError_t launch_insert_remote(const uint64_t* recv_fp, const uint64_t* counts, int nshard, uint64_t cap,
                                uint64_t* table, int tlog2, uint32_t* ans, uint64_t* new_count, DevCounters* ctr,
                                uint64_t max_count, hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_insert_remote, dim3(grid_x(max_count, 256), nshard), dim3(256), 0, st,
                     (const unsigned long long*)recv_fp, (const unsigned long long*)counts, nshard,
                     (unsigned long long)cap, (unsigned long long*)table, tlog2, ans, (unsigned long long*)new_count,
                     ctr);
  return hipGetLastError();
}

hipError_t launch_pack_rows(const Layout& L, const Ring& cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                            const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap, uint64_t lo,
                            uint64_t hi, uint32_t* rows, uint64_t rows_cap, DevCounters* ctr, uint64_t max_count,
                            hipStream_t st) {
  if (!max_count) return hipSuccess;
  const int wpb = std::max(1, expand_lane_wpb(L));
  const size_t lds = (size_t)wpb * lane_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  RTLA_DISPATCH_N(L, k_pack_rows, dim3(grid_x(max_count, 64 * wpb), nshard), dim3(64 * wpb), lds, st, L, cur,
                  (unsigned long long)cur_base, me, (const unsigned long long*)send_ref, ans,
                  (const unsigned long long*)counts, nshard, (unsigned long long)cap, (unsigned long long)lo,
                  (unsigned long long)hi, rows, (unsigned long long)rows_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_unpack_rows(int W, const uint32_t* rows, const uint64_t* counts, const uint64_t* bases, int nshard,
                              uint64_t rows_cap, const Ring& next, uint64_t* parents, uint64_t next_base,
                              uint64_t next_cap, DevCounters* ctr, uint64_t max_count, hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_rows, dim3(grid_x(max_count, 4), nshard), dim3(256), 0, st, W, rows,
                     (const unsigned long long*)counts, (const unsigned long long*)bases, nshard,
                     (unsigned long long)rows_cap, next, (unsigned long long*)parents, (unsigned long long)next_base,
                     (unsigned long long)next_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_part_counts(const uint64_t* new_count, int nshard, uint64_t lo, uint64_t rc, uint64_t* rows_in,
                              uint64_t* bases, DevCounters* ctr, hipStream_t st) {
  hipLaunchKernelGGL(k_part_counts, dim3(1), dim3(64), 0, st, (const unsigned long long*)new_count, nshard,
                     (unsigned long long)lo, (unsigned long long)rc, (unsigned long long*)rows_in,
                     (unsigned long long*)bases, ctr);
  return hipGetLastError();
}

hipError_t launch_insert_rows(const Layout& L, const uint32_t* rows, uint64_t n, uint64_t* table, int tlog2,
                              int* new_flags, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_insert_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, L, rows,
                     (unsigned long long)n, (unsigned long long*)table, tlog2, new_flags, ctr);
  return hipGetLastError();
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

hipError_t launch_random_rows(const Layout& L, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool, uint32_t* out,
                              hipStream_t st) {
  if (!n) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 63) / 64, 256 * 32);
  hipLaunchKernelGGL(k_random_rows, dim3(blocks), dim3(64), (size_t)64 * L.W * sizeof(uint32_t), st, L,
                     (unsigned long long)seed, (unsigned long long)first, (unsigned long long)n,
                     (unsigned long long)pool, out);
  return hipGetLastError();
}

hipError_t launch_probe_bench(uint64_t* table, int tlog2, uint64_t n, uint64_t seed, DevCounters* ctr,
                              hipStream_t st, int load_first) {
  hipLaunchKernelGGL(k_probe_bench, dim3(256 * 16), dim3(256), 0, st, (unsigned long long*)table, tlog2,
                     (unsigned long long)n, (unsigned long long)seed, ctr, load_first);
  return hipGetLastError();
}

}  // namespace rtla
