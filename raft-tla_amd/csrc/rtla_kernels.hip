// rtla_kernels.hip -- gfx950 kernels of the BFS hot path.
//
// One BFS level = one launch of k_expand over the current frontier:
//   * one wavefront per frontier state: the 64 lanes copy the packed row into
//     LDS (coalesced), lane 0 derives the per-parent allLogs' (raft.tla:465);
//   * each lane evaluates one action instance of Next (raft.tla:454-463) as a
//     Delta against the LDS row (rtla_model.h), so every lane reads the same
//     parent words (LDS broadcast, no bank conflicts);
//   * the successor's 128-bit fingerprint is the parent's plus the Delta's
//     component change (no full re-hash);
//   * in-model successors probe the open-addressing fingerprint set in HBM
//     (8-B slots, CAS insert; home slot from fp.a, stored key fp.b | 1);
//   * new successors are compacted by ballot + popcount prefix, built in an
//     LDS staging tile (one row per new lane, odd row stride) and written to
//     the next frontier as one contiguous, coalesced range;
//   * invariants are checked on every new and every out-of-model successor.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rtla_device.h"
#include "rtla_model.h"

using namespace rtla;

namespace {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ unsigned long long shfl0_u64(unsigned long long v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

// Insert into the fingerprint set.  1 = newly inserted, 0 = already present,
// -1 = probe limit exceeded (set too full).  Slots only ever change 0 -> key,
// so a plain read that returns a non-zero value is final; a zero is confirmed
// by the CAS.
__device__ __forceinline__ int fpset_insert(unsigned long long* table, int log2, FP f) {
  const unsigned long long key = f.b | 1ull;
  const unsigned long long mask = (1ull << log2) - 1ull;
  unsigned long long idx = f.a >> (64 - log2);
  for (int probe = 0; probe < 4096; probe++) {
    unsigned long long cur = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return 0;
    if (cur == 0ull) {
      unsigned long long old = atomicCAS(&table[idx], 0ull, key);
      if (old == 0ull) return 1;
      if (old == key) return 0;
    }
    idx = (idx + 1ull) & mask;
  }
  return -1;
}

__device__ __forceinline__ void set_flag(DevCounters* c, int f) { atomicOr(&c->flags, f); }

// Map the q-th candidate of a parent with `nmsg` bag slots to an instance id:
// the fixed families first, then Receive / Duplicate / Drop over used slots.
__device__ __forceinline__ int candidate_inst(const Layout& L, int q, int nmsg) {
  const int fixed = L.fam[F_RECEIVE];
  if (q < fixed) return q;
  int r = q - fixed;
  int fam = r / nmsg, slot = r - fam * nmsg;
  return L.fam[F_RECEIVE + fam] + slot;
}

__device__ __forceinline__ int cover_code(const Layout& L, int inst, int sub) {
  int fam = 0;
  while (fam + 1 < F_COUNT && inst >= L.fam[fam + 1]) fam++;
  return fam == F_RECEIVE ? F_COUNT + sub : fam;
}

}  // namespace

// LDS per wave: parent row (W) + new allLogs words (32) + staging (64 rows x W).
extern "C" __global__ void __launch_bounds__(256)
k_expand(Layout L, const uint32_t* __restrict__ cur, unsigned long long s_begin, unsigned long long s_end,
         unsigned long long cur_base, uint32_t* __restrict__ next,
         unsigned long long* __restrict__ parents, unsigned long long next_base,
         unsigned long long next_cap, unsigned long long* table, int tlog2, DevCounters* ctr,
         ShardBox box) {
  extern __shared__ uint32_t lds[];
  __shared__ unsigned int cov[2 * COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * (W + 32);
  uint32_t* pall = prow + W;
  uint32_t* stage = lds + wpb * (W + 32) + wave * 64 * W;
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();

  unsigned long long my_gen = 0, my_probe = 0;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = s_begin + (unsigned long long)blockIdx.x * wpb + wave; s < s_end;
       s += (unsigned long long)gridDim.x * wpb) {
    const uint32_t* src = cur + s * (unsigned long long)W;
    for (int w = lane; w < W; w += 64) prow[w] = src[w];
    wave_sync();
    FP afp{0, 0};
    if (lane == 0) afp = alllogs_delta(L, prow, pall);
    afp.a = shfl0_u64(afp.a);
    afp.b = shfl0_u64(afp.b);
    wave_sync();
    const FP pfp = fp_add(row_fp(prow), afp);
    const int nmsg = row_nmsg(L, prow);
    const int ncand = fixed + 3 * nmsg;
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      Delta d;
      d.enabled = 0;
      int inst = 0;
      if (q < ncand) {
        inst = candidate_inst(L, q, nmsg);
        compute_delta(L, prow, inst, d);
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
        cfp = fp_add(pfp, delta_fp(L, prow, d));
        const int owner = fp_owner(cfp, box.nshard);
        if (owner == box.me) {
          my_probe++;
          int r = fpset_insert(table, tlog2, cfp);
          if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
          isnew = r == 1;
        } else {
          // Another shard owns this fingerprint: queue (fp, parent, instance);
          // the owner answers new/seen and this shard materialises the winner.
          unsigned long long slot = atomicAdd(&box.out_count[owner], 1ull);
          if (slot < box.cap) {
            unsigned long long k = (unsigned long long)owner * box.cap + slot;
            box.send_fp[2 * k] = cfp.a;
            box.send_fp[2 * k + 1] = cfp.b;
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
        if (isnew) materialize(L, prow, d, pall, cfp, stage + rank * W);
        wave_sync();
        if (obase + cnt <= next_cap) {
          uint32_t* dst = next + obase * (unsigned long long)W;
          for (int w = lane; w < cnt * W; w += 64) dst[w] = stage[w];
          if (isnew)
            parents[next_base + obase + rank] =
                (unsigned long long)box.me << 56 | (cur_base + s) << 16 | (unsigned long long)inst;
        } else if (lane == 0) {
          set_flag(ctr, FLAG_FRONTIER_FULL);
        }
        wave_sync();
      }
      if (en && (isnew || !d.in_model)) {
        int bad = check_invariants(L, prow, &d);
        if (bad && atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
          ctr->viol_parent = cur_base + s;
          ctr->viol_inst = inst;
          ctr->viol_in_model = d.in_model;
          ctr->viol_child = isnew ? next_base + obase + rank : ~0ull;
        }
      }
    }
  }
  // generated: one atomic per wave
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
extern "C" __global__ void k_insert_remote(const unsigned long long* __restrict__ recv_fp,
                                           const unsigned long long* __restrict__ counts, int nshard,
                                           unsigned long long cap, unsigned long long* table, int tlog2,
                                           uint32_t* __restrict__ ans, unsigned long long* __restrict__ new_count,
                                           DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long probes = 0;
  for (; i < (unsigned long long)nshard * cap; i += stride) {
    unsigned long long p = i / cap, k = i - p * cap;
    if (k >= counts[p]) continue;
    FP f{recv_fp[2 * i], recv_fp[2 * i + 1]};
    int r = fpset_insert(table, tlog2, f);
    if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
    ans[i] = r == 1 ? (uint32_t)atomicAdd(&new_count[p], 1ull) + 1u : 0u;
    probes++;
  }
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off);
  if ((threadIdx.x & 63) == 0 && probes) atomicAdd(&ctr->probes, probes);
}

// Sender side: materialise the queued successors whose owner answered "new"
// with a rank in [lo, hi) into the owner's row region (row + parent record,
// RW = W + 2 words per slot).  Invariants are checked here, where parent and
// action are known; a violation is recorded against the local parent.
extern "C" __global__ void k_pack_rows(Layout L, const uint32_t* __restrict__ cur, unsigned long long cur_base,
                                       int me, const unsigned long long* __restrict__ send_ref,
                                       const uint32_t* __restrict__ ans,
                                       const unsigned long long* __restrict__ counts, int nshard,
                                       unsigned long long cap, unsigned long long lo, unsigned long long hi,
                                       uint32_t* __restrict__ rows, unsigned long long rows_cap, DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  const int RW = L.W + 2;
  uint32_t all_new[32];
  for (; i < (unsigned long long)nshard * cap; i += stride) {
    unsigned long long p = i / cap, k = i - p * cap;
    if (k >= counts[p]) continue;
    unsigned long long a = ans[i];
    if (a == 0 || a - 1 < lo || a - 1 >= hi) continue;
    unsigned long long ref = send_ref[i];
    unsigned long long s = ref >> 16;
    int inst = (int)(ref & 0xffff);
    const uint32_t* prow = cur + s * (unsigned long long)L.W;
    Delta d;
    compute_delta(L, prow, inst, d);
    FP afp = alllogs_delta(L, prow, all_new);
    FP cfp = fp_add(fp_add(row_fp(prow), afp), delta_fp(L, prow, d));
    uint32_t* dst = rows + (p * rows_cap + (a - 1 - lo)) * (unsigned long long)RW;
    materialize(L, prow, d, all_new, cfp, dst);
    unsigned long long pr = (unsigned long long)me << 56 | (cur_base + s) << 16 | (unsigned long long)inst;
    dst[L.W] = (uint32_t)pr;
    dst[L.W + 1] = (uint32_t)(pr >> 32);
    int code = cover_code(L, inst, d.sub);
    atomicAdd(&ctr->cover[COVER_CODES + code], 1ull);
    int bad = check_invariants(L, prow, &d);
    if (bad && atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
      ctr->viol_parent = cur_base + s;
      ctr->viol_inst = inst;
      ctr->viol_in_model = 1;
      ctr->viol_child = ~0ull;
    }
  }
}

// Owner side: append the received rows to the next frontier (one wave per
// row, coalesced copy) with their cross-shard parent records.
extern "C" __global__ void k_unpack_rows(int W, const uint32_t* __restrict__ rows,
                                         const unsigned long long* __restrict__ counts, int nshard,
                                         unsigned long long rows_cap, uint32_t* __restrict__ next,
                                         unsigned long long* __restrict__ parents, unsigned long long next_base,
                                         unsigned long long next_cap, DevCounters* ctr) {
  const int lane = threadIdx.x & 63;
  const int RW = W + 2;
  unsigned long long wv = (blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x) >> 6;
  unsigned long long nw = ((unsigned long long)gridDim.x * blockDim.x) >> 6;
  for (unsigned long long i = wv; i < (unsigned long long)nshard * rows_cap; i += nw) {
    unsigned long long p = i / rows_cap, k = i - p * rows_cap;
    if (k >= counts[p]) continue;
    const uint32_t* src = rows + i * (unsigned long long)RW;
    unsigned long long o = 0;
    if (lane == 0) o = atomicAdd(&ctr->next_count, 1ull);
    o = shfl0_u64(o);
    if (o >= next_cap) {
      if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
      continue;
    }
    uint32_t* dst = next + o * (unsigned long long)W;
    for (int w = lane; w < W; w += 64) dst[w] = src[w];
    if (lane == 0) parents[next_base + o] = (unsigned long long)src[W] | (unsigned long long)src[W + 1] << 32;
  }
}

// Insert the fingerprints of `n` rows (Init).  new_flags[i] = 1 if new.
extern "C" __global__ void k_insert_rows(Layout L, const uint32_t* rows, unsigned long long n,
                                         unsigned long long* table, int tlog2, int* new_flags,
                                         DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  FP f = row_fp(rows + (unsigned long long)i * L.W);
  int r = fpset_insert(table, tlog2, f);
  if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
  new_flags[i] = r == 1;
}

// Parity seam: every enabled successor of every input row (in-model or not),
// materialised.  out_info[k] = input index << 32 | in_model << 31 | sub << 16 | inst.
extern "C" __global__ void __launch_bounds__(256)
k_expand_batch(Layout L, const uint32_t* __restrict__ rows, unsigned long long n,
               uint32_t* __restrict__ out, unsigned long long* __restrict__ out_info,
               unsigned long long cap, DevCounters* ctr) {
  extern __shared__ uint32_t lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * (W + 32);
  uint32_t* pall = prow + W;
  uint32_t* stage = lds + wpb * (W + 32) + wave * 64 * W;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wave; s < n;
       s += (unsigned long long)gridDim.x * wpb) {
    for (int w = lane; w < W; w += 64) prow[w] = rows[s * W + w];
    wave_sync();
    FP afp{0, 0};
    if (lane == 0) afp = alllogs_delta(L, prow, pall);
    afp.a = shfl0_u64(afp.a);
    afp.b = shfl0_u64(afp.b);
    wave_sync();
    const FP pfp = fp_add(row_fp(prow), afp);
    const int nmsg = row_nmsg(L, prow);
    const int ncand = fixed + 3 * nmsg;
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      Delta d;
      d.enabled = 0;
      int inst = 0;
      if (q < ncand) {
        inst = candidate_inst(L, q, nmsg);
        compute_delta(L, prow, inst, d);
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
      if (en) materialize(L, prow, d, pall, fp_add(pfp, delta_fp(L, prow, d)), stage + rank * W);
      wave_sync();
      if (obase + cnt <= cap) {
        uint32_t* dst = out + obase * (unsigned long long)W;
        for (int w = lane; w < cnt * W; w += 64) dst[w] = stage[w];
        if (en)
          out_info[obase + rank] = s << 32 | (unsigned long long)(d.in_model ? 1u : 0u) << 31 |
                                   (unsigned long long)d.sub << 16 | (unsigned long long)inst;
      } else if (lane == 0) {
        set_flag(ctr, FLAG_FRONTIER_FULL);
      }
      wave_sync();
    }
  }
}

// Microbenchmark kernel: random 8-B CAS inserts into a table (calibrates the
// random-access roofline of the fingerprint set).
extern "C" __global__ void k_probe_bench(unsigned long long* table, int tlog2, unsigned long long n,
                                         unsigned long long seed, DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long got = 0;
  for (; i < n; i += stride) {
    FP f = hash_u64(seed, i);
    got += fpset_insert(table, tlog2, f) == 1;
  }
  for (int off = 32; off > 0; off >>= 1) got += __shfl_down(got, off);
  if ((threadIdx.x & 63) == 0 && got) atomicAdd(&ctr->next_count, got);
}

// ---------------------------------------------------------------- launch ----
namespace rtla {

size_t expand_lds_bytes(const Layout& L, int wpb) {
  return (size_t)wpb * ((size_t)(L.W + 32) + 64u * (size_t)L.W) * sizeof(uint32_t);
}

int expand_blocks_per_cu(const Layout& L) {
  size_t per = expand_lds_bytes(L, 4) + 2 * COVER_CODES * sizeof(unsigned int);
  int b = (int)((160u * 1024u) / per);
  return b < 1 ? 1 : (b > 8 ? 8 : b);
}

hipError_t launch_expand(const Layout& L, const uint32_t* cur, uint64_t s_begin, uint64_t s_end,
                         uint64_t cur_base, uint32_t* next, uint64_t* parents, uint64_t next_base,
                         uint64_t next_cap, uint64_t* table, int tlog2, DevCounters* ctr, const ShardBox& box,
                         int grid, hipStream_t st) {
  if (s_end <= s_begin) return hipSuccess;
  hipLaunchKernelGGL(k_expand, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, cur,
                     (unsigned long long)s_begin, (unsigned long long)s_end, (unsigned long long)cur_base,
                     next, (unsigned long long*)parents, (unsigned long long)next_base,
                     (unsigned long long)next_cap, (unsigned long long*)table, tlog2, ctr, box);
  return hipGetLastError();
}

hipError_t launch_insert_remote(const uint64_t* recv_fp, const uint64_t* counts, int nshard, uint64_t cap,
                                uint64_t* table, int tlog2, uint32_t* ans, uint64_t* new_count, DevCounters* ctr,
                                hipStream_t st) {
  uint64_t n = (uint64_t)nshard * cap;
  uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_insert_remote, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const unsigned long long*)recv_fp, (const unsigned long long*)counts, nshard,
                     (unsigned long long)cap, (unsigned long long*)table, tlog2, ans,
                     (unsigned long long*)new_count, ctr);
  return hipGetLastError();
}

hipError_t launch_pack_rows(const Layout& L, const uint32_t* cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                            const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap, uint64_t lo,
                            uint64_t hi, uint32_t* rows, uint64_t rows_cap, DevCounters* ctr, hipStream_t st) {
  uint64_t n = (uint64_t)nshard * cap;
  uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)blocks), dim3(256), 0, st, L, cur, (unsigned long long)cur_base, me,
                     (const unsigned long long*)send_ref, ans, (const unsigned long long*)counts, nshard,
                     (unsigned long long)cap, (unsigned long long)lo, (unsigned long long)hi, rows,
                     (unsigned long long)rows_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_unpack_rows(int W, const uint32_t* rows, const uint64_t* counts, int nshard, uint64_t rows_cap,
                              uint32_t* next, uint64_t* parents, uint64_t next_base, uint64_t next_cap,
                              DevCounters* ctr, hipStream_t st) {
  uint64_t waves = (uint64_t)nshard * rows_cap;
  uint64_t blocks = std::min<uint64_t>((waves + 3) / 4, 8192);
  hipLaunchKernelGGL(k_unpack_rows, dim3((unsigned)blocks), dim3(256), 0, st, W, rows,
                     (const unsigned long long*)counts, nshard, (unsigned long long)rows_cap, next,
                     (unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)next_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_insert_rows(const Layout& L, const uint32_t* rows, uint64_t n, uint64_t* table,
                              int tlog2, int* new_flags, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_insert_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, L, rows,
                     (unsigned long long)n, (unsigned long long*)table, tlog2, new_flags, ctr);
  return hipGetLastError();
}

hipError_t launch_expand_batch(const Layout& L, const uint32_t* rows, uint64_t n, uint32_t* out,
                               uint64_t* info, uint64_t cap, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 3) / 4;
  int grid = (int)(blocks < 4096 ? blocks : 4096);
  hipLaunchKernelGGL(k_expand_batch, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, rows,
                     (unsigned long long)n, out, (unsigned long long*)info, (unsigned long long)cap,
                     ctr);
  return hipGetLastError();
}

hipError_t launch_probe_bench(uint64_t* table, int tlog2, uint64_t n, uint64_t seed,
                              DevCounters* ctr, hipStream_t st) {
  hipLaunchKernelGGL(k_probe_bench, dim3(256 * 16), dim3(256), 0, st, (unsigned long long*)table,
                     tlog2, (unsigned long long)n, (unsigned long long)seed, ctr);
  return hipGetLastError();
}

}  // namespace rtla
