// rtla_kwave.hip -- the wave-per-state level kernel k_expand: the fallback
// for rows too wide for k_expand_compact's LDS tile (and RTLA_XFLAGS=2048).
//   * one wavefront per frontier state: the 64 lanes copy the packed row into
//     LDS (coalesced); lanes 0..N-1 hash the parent's server records and lane
//     N derives the per-parent allLogs' (raft.tla:465);
//   * each lane evaluates one action instance of Next (raft.tla:454-463) as a
//     Delta against the LDS row (rtla_model.h);
//   * the successor's 128-bit fingerprint is the parent's plus the Delta's
//     component change; in-model successors CAS-insert into the set;
//   * new successors are compacted by ballot + popcount prefix, built in a
//     16-row LDS staging tile and written to the next frontier coalesced;
//   * invariants are checked on every new and every out-of-model successor.
#include "rtla_kernels_common.h"

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

namespace rtla {

hipError_t launch_wave_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end, uint64_t cur_base,
                              const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap,
                              uint64_t* table, int tlog2, DevCounters* ctr, const ShardBox& box, int grid,
                              hipStream_t st) {
  RTLA_DISPATCH_N(L, k_expand, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, cur,
                  (unsigned long long)s_begin, (unsigned long long)s_end, (unsigned long long)cur_base, next,
                  (unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)next_cap,
                  (unsigned long long*)table, tlog2, ctr, box);
  return hipGetLastError();
}

}  // namespace rtla
