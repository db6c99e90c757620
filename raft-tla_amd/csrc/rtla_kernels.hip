// rtla_kernels.hip -- the level-kernel dispatch and the small kernels of the
// BFS hot path on gfx950.
//
// One BFS level on one shard = one launch of k_expand_compact
// (rtla_kernels_common.h), picked here by layout from
// the instantiation units (rtla_kspec_*, rtla_ksym_*, rtla_kgeneric_*), or of
// the wave-per-state fallback k_expand (rtla_kwave.hip).  This unit also
// holds the multi-shard exchange kernels (k_insert_remote, and the level-end
// re-balancing's k_stage_rows / k_unpack_rows), Init's insert, the synthetic microbench's state generator
// and the fingerprint-set calibration kernel.
#include "rtla_kernels_common.h"

using namespace rtla;

// Owner side of the exchange: insert the fingerprints other shards sent and
// answer each record with 1 (new: the sender builds the state) or 0 (seen).
// Region p holds counts[p] records.  Record slot t of the launch is record
// t / nshard of region t % nshard: the sources interleave, so when several
// senders queued the same new fingerprint in one round, which one wins (and
// builds its row) is not biased towards low shard ids -- the shards' next
// levels stay even without re-balancing.  Each thread takes IR slots a
// stride apart and issues their home-slot loads together (IR random reads
// in flight per lane).
#ifndef RTLA_INSERT_IR
#define RTLA_INSERT_IR 4
#endif
constexpr int IR = RTLA_INSERT_IR;
__global__ void k_insert_remote(const unsigned long long* __restrict__ recv_fp,
                                const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap,
                                unsigned long long max_count, unsigned long long* table, int tlog2,
                                uint32_t* __restrict__ ans, DevCounters* ctr) {
  const int lane = threadIdx.x & 63;
  unsigned probes = 0;
  const unsigned long long total = max_count * (unsigned long long)nshard;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long t0 = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; t0 < total;
       t0 += IR * stride) {
    FP f[IR];
    unsigned long long at[IR];  // p * cap + k, or ~0 (no record)
    unsigned long long seen[IR];
#pragma unroll
    for (int u = 0; u < IR; u++) {
      const unsigned long long t = t0 + u * stride;
      const unsigned long long p = t % (unsigned long long)nshard, k = t / (unsigned long long)nshard;
      at[u] = t < total && k < counts[p] ? p * cap + k : ~0ull;
      f[u] = at[u] != ~0ull ? FP{recv_fp[2 * at[u]], recv_fp[2 * at[u] + 1]} : FP{0, 0};
    }
#pragma unroll
    for (int u = 0; u < IR; u++)  // load first (the owner may know the state: a load is cheaper than an atomic)
      seen[u] = (f[u].a | f[u].b) ? __hip_atomic_load(&table[f[u].a >> (64 - tlog2)], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                  : 0ull;
#pragma unroll
    for (int u = 0; u < IR; u++) {
      if (at[u] == ~0ull) continue;
      uint32_t r = 0;
      if (f[u].a | f[u].b) {  // 0:0 = a hole in the sender's outbox chunk
        r = fpset_resolve_loaded(table, tlog2, f[u].b | 1ull, f[u].a >> (64 - tlog2), seen[u], ctr) ? 1u : 0u;
        probes++;
      }
      ans[at[u]] = r;
    }
  }
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off);
  if (lane == 0 && probes) atomicAdd(&ctr->probes, (unsigned long long)probes);
}

// Exchange round start: the previous round's overflow list (records queued
// past their owner region's end) into this round's outbox regions -- the
// regions are empty, so nearly all fit; what does not goes back on the new
// overflow list.  One record per lane; a wave reserves each owner's slots
// with one atomic.
__global__ void k_requeue(const unsigned long long* __restrict__ in_fp, const unsigned long long* __restrict__ in_ref,
                          const unsigned long long* __restrict__ in_count, ShardBox box, DevCounters* ctr) {
  const unsigned long long n = *in_count;
  const int lane = threadIdx.x & 63;
  const unsigned long long lanes_below = (1ull << lane) - 1ull;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  const unsigned long long start = (unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  for (unsigned long long k0 = start; k0 < n; k0 += stride) {  // (wave-uniform trip count)
    const unsigned long long k = k0 + lane;
    const bool act = k < min(n, box.over_cap);
    const FP f = act ? FP{in_fp[2 * k], in_fp[2 * k + 1]} : FP{0, 0};
    const unsigned long long ref = act ? in_ref[k] : 0ull;
    const int o = act ? fp_owner(f, box.nshard) : -1;
    unsigned long long slot = ~0ull;
    for (int p = 0; p < box.nshard; p++) {
      const unsigned long long m = __ballot(o == p);
      if (!m) continue;
      unsigned long long b = 0;
      if (lane == __builtin_ctzll(m)) b = atomicAdd(&box.out_count[p], (unsigned long long)__popcll(m));
      b = shfl_u64(b, __builtin_ctzll(m));
      if (o == p) slot = b + __popcll(m & lanes_below);
    }
    if (act && slot < box.cap) {
      const unsigned long long q = (unsigned long long)o * box.cap + slot;
      box.send_fp[2 * q] = f.a;
      box.send_fp[2 * q + 1] = f.b;
      box.send_ref[q] = ref;
    }
    const bool ov = act && slot >= box.cap;
    const unsigned long long om = __ballot(ov);
    if (om) {
      unsigned long long ob = 0;
      if (lane == 0) ob = atomicAdd(box.over_count, (unsigned long long)__popcll(om));
      ob = shfl0_u64(ob);
      if (ov) {
        const unsigned long long q = ob + __popcll(om & lanes_below);
        if (q < box.over_cap) {
          box.over_fp[2 * q] = f.a;
          box.over_fp[2 * q + 1] = f.b;
          box.over_ref[q] = ref;
        } else {
          set_flag(ctr, FLAG_OUTBOX_FULL);
        }
      }
    }
  }
}

// Exchange round end, on the device (read back by the round's one count
// gather): how much of the frontier range the level kernel left, and the
// overflow list's length.
__global__ void k_round_tail(const DevCounters* ctr, unsigned long long* out, int G, unsigned long long span,
                             unsigned long long rest, int grouped, const unsigned long long* over_count) {
  if (threadIdx.x != 0) return;
  unsigned long long done = span;
  if (grouped) done = min(span, ctr->group_next * ctr->group_size);
  out[G] = rest + span - done;
  out[G + 1] = over_count ? *over_count : 0ull;
}

// Re-balancing, receiving side: append the staged rows to the next frontier
// (one wave per row, coalesced copy) with their parent records.
__global__ void k_unpack_rows(int W, const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ counts,
                              const unsigned long long* __restrict__ bases, int nshard, unsigned long long rows_cap,
                              Ring next, unsigned long long* __restrict__ parents,
                              unsigned long long next_base, unsigned long long next_cap, DevCounters* ctr) {
  // grid.y = source shard p; its rows land at the contiguous slots bases[p] + k
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

// Re-balancing (rtla_step, level end): copy states [first, first + n) of a
// shard's next level -- rows and parent records -- into a staging region of
// n slots of W + 2 words (the k_unpack_rows format), one wave per row.
__global__ void k_stage_rows(int W, Ring next, const unsigned long long* __restrict__ parents,
                             unsigned long long next_base, unsigned long long first, unsigned long long n,
                             uint32_t* __restrict__ rows) {
  const int lane = threadIdx.x & 63;
  const int RW = W + 2;
  const unsigned long long wv = (blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x) >> 6;
  const unsigned long long nw = ((unsigned long long)gridDim.x * blockDim.x) >> 6;
  for (unsigned long long k = wv; k < n; k += nw) {
    const uint32_t* src = ring_row(next, first + k, W);
    uint32_t* dst = rows + k * (unsigned long long)RW;
    for (int w = lane; w < W; w += 64) dst[w] = src[w];
    if (lane == 0) {
      const unsigned long long pr = parents[next_base + first + k];
      dst[W] = (uint32_t)pr;
      dst[W + 1] = (uint32_t)(pr >> 32);
    }
  }
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

// Mixed-stream calibration (bench.py's random-access ceiling): probe i is,
// with probability new_frac (threshold q of 2^64), a key never inserted
// before, else one of the n_present keys inserted beforehand -- the level
// kernel's protocol on each: load the home slot, CAS only when it reads
// empty (linear probing on).  ctr->next_count counts the inserts.
__global__ void k_probe_mixed(unsigned long long* table, int tlog2, unsigned long long n, unsigned long long n_present,
                              unsigned long long q, unsigned long long seed, DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long got = 0;
  for (; i < n; i += stride) {
    const FP pick = hash_u64(seed ^ 0x6d69786564ull, i);
    const FP f = pick.a < q ? hash_u64(seed + 1, i) : hash_u64(seed, pick.b % n_present);
    const unsigned long long idx = f.a >> (64 - tlog2);
    const unsigned long long v = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    got += fpset_resolve_loaded(table, tlog2, f.b | 1ull, idx, v, ctr) ? 1 : 0;
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

hipError_t launch_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end, uint64_t cur_base,
                         const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap, uint64_t* table,
                         int tlog2, DevCounters* ctr, const ShardBox& box, int grid, hipStream_t st, int xflags,
                         uint64_t* sent, hipEvent_t mid) {
  if (s_end <= s_begin) return hipSuccess;
  const int cwpb = expand_compact_wpb(L);
  if (cwpb > 0 && !(xflags & XF_WAVE_KERNEL)) {
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
    if (!done && L.sym) e = launch_compact_sym_a(a, &done);
    if (!done && L.sym) e = launch_compact_sym_b(a, &done);
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
  return launch_wave_expand(L, cur, s_begin, s_end, cur_base, next, parents, next_base, next_cap, table, tlog2, ctr,
                            box, grid, st);
}

bool level_kernel_shape(const Layout& L, bool multi, int xflags, int* waves, int* group) {
  *waves = 0;
  *group = 0;
  if (expand_compact_wpb(L) <= 0 || (xflags & XF_WAVE_KERNEL)) return false;
  int q[2] = {0, 0};
  CompactArgs a{};
  a.L = L;
  a.multi = multi;
  a.s_begin = 0;
  a.s_end = 64;
  a.xflags = xflags;
  a.wpb = (xflags & XF_BLOCK4) ? expand_compact_wpb(L) : 1;
  a.box.nshard = multi ? 2 : 1;
  a.query = q;
  bool done = false;
  if (!(xflags & XF_NO_SPECIAL)) {
    (void)launch_compact_spec_a(a, &done);
    if (!done) (void)launch_compact_spec_b(a, &done);
  }
#ifndef RTLA_EXP_MINIMAL
  if (!done && L.sym) (void)launch_compact_sym_a(a, &done);
  if (!done && L.sym) (void)launch_compact_sym_b(a, &done);
  if (!done) (void)launch_compact_generic_a(a, &done);
  if (!done) (void)launch_compact_generic_b(a, &done);
#endif
  if (!done || q[0] <= 0 || q[1] <= 0) return false;
  *waves = q[0];
  *group = q[1];
  return true;
}

hipError_t launch_requeue(const uint64_t* in_fp, const uint64_t* in_ref, const uint64_t* in_count, uint64_t max_count,
                          const ShardBox& box, DevCounters* ctr, hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_requeue, dim3(grid_x(max_count, 256)), dim3(256), 0, st, (const unsigned long long*)in_fp,
                     (const unsigned long long*)in_ref, (const unsigned long long*)in_count, box, ctr);
  return hipGetLastError();
}

hipError_t launch_round_tail(const DevCounters* ctr, uint64_t* out, int G, uint64_t span, uint64_t rest, bool grouped,
                             const uint64_t* over_count, hipStream_t st) {
  hipLaunchKernelGGL(k_round_tail, dim3(1), dim3(64), 0, st, ctr, (unsigned long long*)out, G,
                     (unsigned long long)span, (unsigned long long)rest, grouped ? 1 : 0,
                     (const unsigned long long*)over_count);
  return hipGetLastError();
}

hipError_t launch_insert_remote(const uint64_t* recv_fp, const uint64_t* counts, int nshard, uint64_t cap,
                                uint64_t* table, int tlog2, uint32_t* ans, DevCounters* ctr, uint64_t max_count,
                                hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_insert_remote, dim3(grid_x((max_count * nshard + IR - 1) / IR, 256)), dim3(256), 0, st,
                     (const unsigned long long*)recv_fp, (const unsigned long long*)counts, nshard,
                     (unsigned long long)cap, (unsigned long long)max_count, (unsigned long long*)table, tlog2, ans,
                     ctr);
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

hipError_t launch_stage_rows(int W, const Ring& next, const uint64_t* parents, uint64_t next_base, uint64_t first,
                             uint64_t n, uint32_t* rows, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_stage_rows, dim3(grid_x(n, 4)), dim3(256), 0, st, W, next,
                     (const unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)first,
                     (unsigned long long)n, rows);
  return hipGetLastError();
}

hipError_t launch_insert_rows(const Layout& L, const uint32_t* rows, uint64_t n, uint64_t* table, int tlog2,
                              int* new_flags, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_insert_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, L, rows,
                     (unsigned long long)n, (unsigned long long*)table, tlog2, new_flags, ctr);
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

hipError_t launch_probe_mixed(uint64_t* table, int tlog2, uint64_t n, uint64_t n_present, double new_frac,
                              uint64_t seed, DevCounters* ctr, hipStream_t st) {
  const double qf = std::min(1.0, std::max(0.0, new_frac)) * 18446744073709551616.0;
  const unsigned long long q = qf >= 18446744073709551615.0 ? ~0ull : (unsigned long long)qf;
  hipLaunchKernelGGL(k_probe_mixed, dim3(256 * 16), dim3(256), 0, st, (unsigned long long*)table, tlog2,
                     (unsigned long long)n, (unsigned long long)std::max<uint64_t>(n_present, 1), q,
                     (unsigned long long)seed, ctr);
  return hipGetLastError();
}

}  // namespace rtla
