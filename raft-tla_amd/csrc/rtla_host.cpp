// rtla_host.cpp -- the C-ABI driver (include/rtla.h) around the HIP kernels.
//
// A context owns one or more SHARDS.  A shard is the unit of fingerprint
// ownership: it holds the part of the fingerprint set whose fingerprints it
// owns (fp_owner, rtla_device.h), the states it materialised (frontier double
// buffer) and their parent pointers.  Device memory per shard:
//   fingerprint set   2^fpset_log2 x 8 B   (open addressing, CAS insert)
//   parents           one u64 per state: parent shard << 56 | parent index << 16 | instance
//   row arena         frontier_cap rows (a multiple of 64), used as a ring: the
//                     current level's rows, then the next level's after them
//   outbox / inbox    (multi-shard only) per destination: fingerprints, refs, answers
//
// Deployments:
//   world == 1, shards <= 1 : the whole search in one shard; one fused k_expand
//                             launch per BFS level (expand + probe + insert +
//                             materialise + invariants).
//   world == N (one process per GPU, RCCL over xGMI): one shard per rank.
//   world == 1, shards == S : S shards on one GPU, exchanging by device copies
//                             -- the multi-GPU protocol exercised on one device;
//                             with RTLA_TRANSPORT=rccl the same exchange runs
//                             through a one-rank RCCL communicator instead
//                             (every ncclSend/ncclRecv to self, the count
//                             all-gathers, the level all-reduces, the trace
//                             broadcasts): the RCCL call sites of the
//                             multi-GPU path execute on a one-GPU box.
//
// Multi-shard level: exchange rounds, all shards in lock-step (rtla_step):
//   1. k_expand_compact: successors owned locally are probed, inserted and
//      built at once; the others are queued as (fingerprint, parent ref) per
//      owner.  The kernel expands the rest of the frontier until an owner's
//      outbox region fills (its group guard), so a round is as large as the
//      outbox allows;
//   2. all-gather of the per-owner counts (+ what each shard has left) --
//      the round's only host synchronisation -- then all-to-all-v of the
//      16-byte fingerprints (ncclSend/ncclRecv pairs in one group: all 7 xGMI
//      links of an MI355X node carry traffic at once);
//   3. k_insert_remote at the owner answers each record new / seen;
//   4. all-to-all-v of the answers back;
//   5. k_build_winners: each sender builds the rows of its winners into its
//      own next level (rows never cross shards; parent records name the
//      parent's shard, so traces walk across shards).
// Then one all-reduce of {new, generated, probes, violation, flags} decides
// termination (TLC's "0 states left on queue"), and the next levels are
// re-balanced where they drifted from an even split.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtla.h"
#include "rtla_device.h"
#include "rtla_launch.h"
#include "rtla_model.h"
#include "rtla_synth.h"
#include "rtla_text.h"

using namespace rtla;

namespace {

struct Shard {
  int id = 0;
  uint64_t* table = nullptr;
  uint64_t* parents = nullptr;
  uint64_t parents_cap = 0;
  uint32_t* arena = nullptr;        // frontier rows: the current and the next level, as a ring (Ring)
  uint64_t cur_start = 0;           // arena row of the current level's first state (a multiple of 64)
  uint64_t n_cur = 0, cur_base = 0;
  DevCounters* ctr = nullptr;
  int* dflags = nullptr;
  // exchange buffers (nshard > 1)
  uint64_t* out_count = nullptr;   // [G + 2] device: records queued per destination (reserved slots; those past
                                   // box_cap are on the overflow list), frontier states left, overflow records
  uint64_t* in_count = nullptr;    // [G] device: records received per source
  uint64_t* all_count = nullptr;   // [G][G + 2] device (RCCL all-gather target)
  uint64_t* send_fp = nullptr;     // [G][cap][2]
  uint64_t* send_ref = nullptr;    // [G][cap]
  uint32_t* send_ans = nullptr;    // [G][cap]  owners' answers to our records
  uint64_t* recv_fp = nullptr;     // [G][cap][2]
  uint32_t* recv_ans = nullptr;    // [G][cap]  our answers to the senders
  uint64_t* rows_in = nullptr;     // [G] device: rows received per source (re-balancing sub-round)
  uint64_t* rows_base = nullptr;   // [G] device: next-frontier slot of each source's first row
  uint32_t* send_rows = nullptr;   // [G][rows_cap][W + 2]  re-balancing staging
  uint32_t* recv_rows = nullptr;   // [G][rows_cap][W + 2]
  uint64_t* sent = nullptr;        // [2^slog2] sent cache: fingerprints this shard already sent to their owners
  uint64_t* over_fp[2] = {nullptr, nullptr};   // overflow lists [over_cap][2]: records past their region's end,
  uint64_t* over_ref[2] = {nullptr, nullptr};  // sent in the next round (k_requeue)
  uint64_t* over_cnt = nullptr;    // [2] their lengths
  int ov = 0;                      // the list the next round requeues
  uint64_t pos = 0, over_n = 0;    // this level: next frontier state to expand, records on list ov
  std::vector<uint64_t> h_out, h_in, h_all;
  uint64_t h_reb[2 * SHARD_MAX] = {};  // re-balancing: rows_in / rows_base of this sub-round (host staging)
  uint64_t h_caps[3] = {0, 0, 0};  // -> DevCounters cap_cur / cap_next / cap_parents
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evm = nullptr;
  // violation found on this shard
  int viol_mask = 0, viol_in_model = 0, viol_inst = -1;
  uint64_t viol_parent = 0, viol_child = ~0ull;
};

}  // namespace

// Host shared-memory transport for world > 1 (RTLA_TRANSPORT=shm): the same
// collectives as the RCCL path, staged through a POSIX shared-memory segment
// named after the communicator id.  It lets N processes on ONE GPU run the
// multi-rank protocol -- RCCL refuses two ranks on one device -- so the
// world > 1 control flow (count gathers, all-to-all-v, answer routing,
// reductions, trace broadcasts, recovery checks) is tested on single-GPU
// boxes.  Not a performance path: every operation synchronises the stream.
struct ShmComm {
  struct Header {
    std::atomic<uint32_t> arrive, gen;
    std::atomic<uint32_t> abort;  // a rank failed inside a collective: every wait ends (RTLA_E_COMM)
  };
  Header* hdr = nullptr;
  uint8_t* data = nullptr;   // world x world slots of `slot` bytes: [src][dst]
  size_t slot = 0, size = 0;
  uint8_t* slot_at(int src, int dst, int world) const { return data + ((size_t)src * world + dst) * slot; }
};

struct rtla_ctx {
  rtla_cfg cfg;
  Layout L;
  int rank = 0, world = 1, device = 0;
  int nshard = 1;          // shards in the whole job
  int shard0 = 0;          // global id of sh[0]
  std::vector<Shard> sh;   // shards held by this process
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  ShmComm* shm = nullptr;  // RTLA_TRANSPORT=shm instead of RCCL
  bool rccl_local = false; // world 1, S shards, RTLA_TRANSPORT=rccl: the exchange goes through `comm` (1 rank)
  int tlog2 = 0;
  int slog2 = 0;           // sent cache: 2^slog2 slots per shard (multi-shard)
  uint64_t front_cap = 0, box_cap = 0, chunk = 0, rows_cap = 0;
  uint64_t stop_at = 0, over_cap = 0;  // multi-shard outbox: the level kernel's group guard, overflow list capacity
  bool guarded = false;    // multi-shard rounds run the grouped level kernel (rounds sized by the outbox)
  std::vector<uint64_t> h_rows;  // [G][G + 2] the round's gathered counts, every shard's row
  uint64_t rebalanced = 0; // rows moved by level-end re-balancing (all levels, this process's shards)
  uint64_t rounds = 0;     // exchange rounds run (all levels)
  uint64_t overflowed = 0; // records that went through the overflow list (all levels, this process's shards)
  uint64_t records = 0;    // fingerprint records this process's shards sent to other shards (all levels)
  uint64_t* red = nullptr;  // device scratch for all-reduces
  int level = 0;
  bool inited = false, finished = false;
  uint64_t distinct = 0, generated = 0;
  uint64_t max_front = 0;  // largest frontier of any shard in the job (multi-shard round count)
  int grid = 0;
  std::vector<uint32_t> init_row;
};

// ---- the row arena as a ring (Ring, rtla_device.h)
static uint64_t round64(uint64_t n) { return (n + 63) & ~63ull; }
static Ring cur_ring(const rtla_ctx* x, const Shard& s) { return Ring{s.arena, s.cur_start, x->front_cap}; }
// The next level starts at the first 64-row boundary past the current one
// and may use every arena row the current level does not.
static Ring next_ring(const rtla_ctx* x, const Shard& s) {
  return Ring{s.arena, (s.cur_start + round64(s.n_cur)) % x->front_cap, x->front_cap};
}
static uint64_t next_room(const rtla_ctx* x, const Shard& s) {
  const uint64_t used = round64(s.n_cur);
  return x->front_cap > used ? x->front_cap - used : 0;
}
// Copy states [g, g + n) of a level to / from the host (two pieces if they wrap).
static hipError_t ring_copy(const Ring& r, int W, uint64_t g, uint64_t n, uint32_t* host, bool to_host) {
  while (n) {
    const uint64_t p = ring_idx(r, g), m = std::min<uint64_t>(n, r.cap - p);
    uint32_t* dev = r.base + p * (uint64_t)W;
    hipError_t e = to_host ? hipMemcpy(host, dev, m * W * 4, hipMemcpyDeviceToHost)
                           : hipMemcpy(dev, host, m * W * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) return e;
    host += m * (uint64_t)W;
    g += m;
    n -= m;
  }
  return hipSuccess;
}

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      fprintf(stderr, "rtla: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return RTLA_E_HIP;                                                                            \
    }                                                                                               \
  } while (0)

#define NCCLCHK(x)                                                                                    \
  do {                                                                                                \
    ncclResult_t r_ = (x);                                                                            \
    if (r_ != ncclSuccess) {                                                                          \
      fprintf(stderr, "rtla: RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      return RTLA_E_COMM;                                                                             \
    }                                                                                                 \
  } while (0)

// ---- collectives between ranks: RCCL, or the shared-memory transport (ShmComm)
// Every function is called by every rank in the same order; device buffers,
// in stream order.

static int shm_barrier(rtla_ctx* x) {
  ShmComm::Header* h = x->shm->hdr;
  if (h->abort.load(std::memory_order_acquire)) return RTLA_E_COMM;
  const uint32_t g = h->gen.load(std::memory_order_acquire);
  if (h->arrive.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)x->world - 1) {
    h->arrive.store(0, std::memory_order_relaxed);
    h->gen.fetch_add(1, std::memory_order_acq_rel);
    return RTLA_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  while (h->gen.load(std::memory_order_acquire) == g) {
    if (h->abort.load(std::memory_order_acquire)) {
      fprintf(stderr, "rtla: shm transport: another rank failed inside a collective\n");
      return RTLA_E_COMM;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600)) {
      fprintf(stderr, "rtla: shm transport: the other ranks did not arrive\n");
      return RTLA_E_COMM;
    }
    sched_yield();
  }
  return RTLA_OK;
}

static int shm_open_comm(rtla_ctx* x, const void* comm_id) {
  const uint8_t* id = static_cast<const uint8_t*>(comm_id);
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the 128-byte id
  for (int i = 0; i < 128; i++) h = (h ^ id[i]) * 1099511628211ull;
  char name[64];
  snprintf(name, sizeof name, "/rtla_%016llx", (unsigned long long)h);
  const char* e = getenv("RTLA_SHM_SLOT_MB");
  const size_t slot = (size_t)(e && atoi(e) > 0 ? atoi(e) : 64) << 20;
  const size_t size = 4096 + (size_t)x->world * x->world * slot;
  const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0) return RTLA_E_COMM;
  if (ftruncate(fd, (off_t)size) != 0) {
    close(fd);
    return RTLA_E_COMM;
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return RTLA_E_COMM;
  x->shm = new ShmComm();
  x->shm->hdr = static_cast<ShmComm::Header*>(p);
  x->shm->data = static_cast<uint8_t*>(p) + 4096;
  x->shm->slot = slot;
  x->shm->size = size;
  const int rc = shm_barrier(x);  // every rank has the segment mapped: the name can go
  if (x->rank == 0) shm_unlink(name);
  return rc;
}

static int shm_fail(const ShmComm& c, int rc) {  // a local failure inside a collective: the peers' waits end too
  c.hdr->abort.store(1, std::memory_order_release);
  return rc;
}

static int shm_too_big(size_t bytes, const ShmComm& c) {
  if (bytes <= c.slot) return RTLA_OK;
  fprintf(stderr, "rtla: shm transport: %zu-byte message exceeds the %zu-byte slot (RTLA_SHM_SLOT_MB)\n", bytes, c.slot);
  return shm_fail(c, RTLA_E_COMM);
}

// A HIP call inside an shm collective: on failure mark the abort before returning.
#define SHMCHK(c, x)                                                                                \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      fprintf(stderr, "rtla: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return shm_fail((c), RTLA_E_HIP);                                                             \
    }                                                                                               \
  } while (0)

static int nccl_fail(ncclResult_t r, int line) {
  fprintf(stderr, "rtla: RCCL error %s at %s:%d\n", ncclGetErrorString(r), __FILE__, line);
  return RTLA_E_COMM;
}

// In place: sum (op 0) or max (op 1) of n u64 over all ranks.
static int comm_allreduce(rtla_ctx* x, uint64_t* buf, int n, int op) {
  if (!x->shm) {
    const ncclResult_t r = ncclAllReduce(buf, buf, n, ncclUint64, op ? ncclMax : ncclSum, x->comm, x->stream);
    return r == ncclSuccess ? RTLA_OK : nccl_fail(r, __LINE__);
  }
  const ShmComm& c = *x->shm;
  if (int rc = shm_too_big(8 * (size_t)n, c)) return rc;
  SHMCHK(c, hipMemcpyAsync(c.slot_at(x->rank, 0, x->world), buf, 8 * n, hipMemcpyDeviceToHost, x->stream));
  SHMCHK(c, hipStreamSynchronize(x->stream));
  if (int rc = shm_barrier(x)) return rc;
  std::vector<uint64_t> acc(n, 0);
  for (int r = 0; r < x->world; r++) {
    const uint64_t* v = reinterpret_cast<const uint64_t*>(c.slot_at(r, 0, x->world));
    for (int i = 0; i < n; i++) acc[i] = op ? std::max(acc[i], v[i]) : acc[i] + v[i];
  }
  if (int rc = shm_barrier(x)) return rc;
  SHMCHK(c, hipMemcpyAsync(buf, acc.data(), 8 * n, hipMemcpyHostToDevice, x->stream));
  SHMCHK(c, hipStreamSynchronize(x->stream));
  return RTLA_OK;
}

// recv[r * n + i] = send[i] of rank r.
static int comm_allgather(rtla_ctx* x, const uint64_t* send, uint64_t* recv, int n) {
  if (!x->shm) {
    const ncclResult_t r = ncclAllGather(send, recv, n, ncclUint64, x->comm, x->stream);
    return r == ncclSuccess ? RTLA_OK : nccl_fail(r, __LINE__);
  }
  const ShmComm& c = *x->shm;
  if (int rc = shm_too_big(8 * (size_t)n, c)) return rc;
  SHMCHK(c, hipMemcpyAsync(c.slot_at(x->rank, 0, x->world), send, 8 * n, hipMemcpyDeviceToHost, x->stream));
  SHMCHK(c, hipStreamSynchronize(x->stream));
  if (int rc = shm_barrier(x)) return rc;
  for (int r = 0; r < x->world; r++)
    SHMCHK(c, hipMemcpyAsync(recv + (size_t)r * n, c.slot_at(r, 0, x->world), 8 * n, hipMemcpyHostToDevice, x->stream));
  SHMCHK(c, hipStreamSynchronize(x->stream));
  return shm_barrier(x);
}

static int comm_bcast(rtla_ctx* x, uint64_t* buf, int n, int root) {
  if (!x->shm) {
    const ncclResult_t r = ncclBroadcast(buf, buf, n, ncclUint64, root, x->comm, x->stream);
    return r == ncclSuccess ? RTLA_OK : nccl_fail(r, __LINE__);
  }
  const ShmComm& c = *x->shm;
  if (int rc = shm_too_big(8 * (size_t)n, c)) return rc;
  if (x->rank == root) {
    SHMCHK(c, hipMemcpyAsync(c.slot_at(root, 0, x->world), buf, 8 * n, hipMemcpyDeviceToHost, x->stream));
    SHMCHK(c, hipStreamSynchronize(x->stream));
  }
  if (int rc = shm_barrier(x)) return rc;
  if (x->rank != root) {
    SHMCHK(c, hipMemcpyAsync(buf, c.slot_at(root, 0, x->world), 8 * n, hipMemcpyHostToDevice, x->stream));
    SHMCHK(c, hipStreamSynchronize(x->stream));
  }
  return shm_barrier(x);
}

// One all-to-all-v round: point-to-point messages (at most one send and one
// receive per peer), all in flight together (one RCCL group).  The group is
// always closed, also when a send or receive could not be posted.
struct Msg {
  void* ptr;
  size_t bytes;
  int peer;
};
static int comm_exchange(rtla_ctx* x, const std::vector<Msg>& sends, const std::vector<Msg>& recvs) {
  if (!x->shm) {
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(r, __LINE__);
    for (const Msg& m : sends)
      if (r == ncclSuccess) r = ncclSend(m.ptr, m.bytes, ncclUint8, m.peer, x->comm, x->stream);
    for (const Msg& m : recvs)
      if (r == ncclSuccess) r = ncclRecv(m.ptr, m.bytes, ncclUint8, m.peer, x->comm, x->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    return r == ncclSuccess ? RTLA_OK : nccl_fail(r, __LINE__);
  }
  const ShmComm& c = *x->shm;
  for (const Msg& m : sends) {
    if (int rc = shm_too_big(m.bytes, c)) return rc;
    SHMCHK(c, hipMemcpyAsync(c.slot_at(x->rank, m.peer, x->world), m.ptr, m.bytes, hipMemcpyDeviceToHost, x->stream));
  }
  SHMCHK(c, hipStreamSynchronize(x->stream));
  if (int rc = shm_barrier(x)) return rc;
  for (const Msg& m : recvs) {
    if (int rc = shm_too_big(m.bytes, c)) return rc;
    SHMCHK(c, hipMemcpyAsync(m.ptr, c.slot_at(m.peer, x->rank, x->world), m.bytes, hipMemcpyHostToDevice, x->stream));
  }
  SHMCHK(c, hipStreamSynchronize(x->stream));
  return shm_barrier(x);
}

// RCCL prints its version banner on stdout when a communicator is created;
// stdout belongs to the caller (the CLI's TLC-format output, bench.py's JSON
// line), so the banner is sent to stderr.
struct StdoutToStderr {
  int saved = -1;
  StdoutToStderr() {
    fflush(stdout);
    saved = dup(1);
    if (saved >= 0) dup2(2, 1);
  }
  ~StdoutToStderr() {
    fflush(stdout);
    if (saved >= 0) {
      dup2(saved, 1);
      close(saved);
    }
  }
};

static int layout_from_cfg(const rtla_cfg* c, Layout* L) {
  if (!c) return RTLA_E_ARG;
  int K = c->bag_cap ? c->bag_cap : (c->max_msgs > 0 ? c->max_msgs + 1 : 32);
  int E = c->elec_cap ? c->elec_cap : (c->max_term - 1) * c->n_server;
  if (E < 1) E = 1;
  if (make_layout(L, c->n_server, c->n_value, c->max_term, c->max_log, c->max_copies, c->max_msgs, K, E,
                  c->inv_mask) != 0)
    return RTLA_E_CONFIG;
  L->sym = c->symmetry ? 1 : 0;
  return RTLA_OK;
}

extern "C" int rtla_abi_version(void) { return RTLA_ABI_VERSION; }

extern "C" const char* rtla_strerror(int s) {
  switch (s) {
    case RTLA_OK: return "ok";
    case RTLA_DONE: return "search complete";
    case RTLA_VIOLATION: return "invariant violated";
    case RTLA_E_CONFIG: return "configuration outside the supported row format";
    case RTLA_E_HIP: return "HIP runtime error";
    case RTLA_E_OVERFLOW: return "capacity overflow (bag/elections/frontier/fingerprint set/outbox)";
    case RTLA_E_SPEC: return "TLC evaluation error in Next (index outside DOMAIN)";
    case RTLA_E_STATE: return "call out of order";
    case RTLA_E_ARG: return "bad argument";
    case RTLA_E_COMM: return "RCCL error";
    default: return "unknown status";
  }
}

extern "C" int rtla_row_words(const rtla_cfg* c) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  return r ? r : L.W;
}

extern "C" int rtla_row_layout(const rtla_cfg* c, int32_t* out, int n) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!out) return RTLA_E_ARG;
  const int32_t v[10] = {L.W, L.off_hdr, L.off_srv, L.srv_w, L.off_all, L.all_words, L.off_elec, L.elec_w, L.off_bag,
                         L.slot_w};
  const int m = std::min(n, 10);
  for (int k = 0; k < m; k++) out[k] = v[k];
  return m;
}

extern "C" int rtla_init_row(const rtla_cfg* c, uint32_t* row) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  row_init(L, row);
  return RTLA_OK;
}

extern "C" int rtla_invariants(const rtla_cfg* c, const uint32_t* row) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  return check_invariants<0>(L, row, (const Delta*)nullptr);
}

extern "C" int rtla_row_fingerprint(const rtla_cfg* c, const uint32_t* row, uint64_t out[2]) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  FP f = row_fingerprint(L, row);
  out[0] = f.a;
  out[1] = f.b;
  return RTLA_OK;
}

extern "C" int rtla_orbit_key(const rtla_cfg* c, const uint32_t* row, uint64_t out[2], int* perms) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  FP f{0, 0};
  switch (L.N) {
    case 1: f = orbit_key_row<1>(L, row, perms); break;
    case 2: f = orbit_key_row<2>(L, row, perms); break;
    case 3: f = orbit_key_row<3>(L, row, perms); break;
    case 4: f = orbit_key_row<4>(L, row, perms); break;
    default: f = orbit_key_row<5>(L, row, perms); break;
  }
  out[0] = f.a;
  out[1] = f.b;
  return RTLA_OK;
}

extern "C" int rtla_permute_row(const rtla_cfg* c, const uint32_t* row, const int* pi, uint32_t* out) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  int seen = 0;
  for (int i = 0; i < L.N; i++) {
    if (pi[i] < 0 || pi[i] >= L.N || (seen >> pi[i] & 1)) return RTLA_E_ARG;
    seen |= 1 << pi[i];
  }
  switch (L.N) {
    case 1: permute_row<1>(L, row, pi, out); break;
    case 2: permute_row<2>(L, row, pi, out); break;
    case 3: permute_row<3>(L, row, pi, out); break;
    case 4: permute_row<4>(L, row, pi, out); break;
    default: permute_row<5>(L, row, pi, out); break;
  }
  return RTLA_OK;
}

extern "C" int rtla_state_text(const rtla_cfg* c, const uint32_t* row, char* buf, size_t cap) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  std::string s = state_text(L, row);
  if (s.size() + 1 > cap) return RTLA_E_ARG;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

extern "C" int rtla_action_name(const rtla_cfg* c, int32_t inst, int32_t sub, char* buf, size_t cap) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  std::string s = action_name(L, inst, sub);
  if (s.size() + 1 > cap) return RTLA_E_ARG;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

// ---- level digests (rtla_rows_text_hash / rtla_level_text_hash): the sum of
// FNV-1a-64 of each state's canonical text, computed by a pool of host threads.
static int text_threads(int want) {
  if (want > 0) return std::min(want, 256);
  int n = 0;
  if (const char* e = getenv("OMP_NUM_THREADS")) n = atoi(e);  // the GPU box's per-job CPU allowance
  if (n <= 0) {
    cpu_set_t cs;
    n = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 8;
  }
  return std::max(1, std::min(n, 16));
}

// FNV-1a is one serial multiply chain per text: 8 texts are hashed together
// so the chains overlap (multiplier throughput, not latency, bounds a core).
constexpr int TEXT_ILP = 8;
static uint64_t fnv1a64_sum(char* const* txt, const size_t* len, int m) {
  uint64_t h[TEXT_ILP];
  size_t common = ~(size_t)0;
  for (int i = 0; i < m; i++) {
    h[i] = 0xcbf29ce484222325ull;
    common = std::min(common, len[i]);
  }
  for (size_t k = 0; k < common; k++)
    for (int i = 0; i < TEXT_ILP; i++)
      if (i < m) h[i] = (h[i] ^ (unsigned char)txt[i][k]) * 0x100000001b3ull;
  uint64_t sum = 0;
  for (int i = 0; i < m; i++) {
    for (size_t k = common; k < len[i]; k++) h[i] = (h[i] ^ (unsigned char)txt[i][k]) * 0x100000001b3ull;
    sum += h[i];
  }
  return sum;
}

static uint64_t rows_digest(const Layout& L, const uint32_t* rows, size_t n, int threads, bool orbit = false) {
  threads = (int)std::min<size_t>((size_t)threads, std::max<size_t>(1, n / 4096));
  std::vector<uint64_t> part((size_t)threads, 0);
  std::atomic<size_t> next{0};
  const size_t cap = state_text_cap(L);
  auto work = [&](int t) {
    std::vector<char> buf((TEXT_ILP + 1) * cap);  // TEXT_ILP texts + one scratch area
    char* txt[TEXT_ILP];
    size_t len[TEXT_ILP];
    for (int i = 0; i < TEXT_ILP; i++) txt[i] = buf.data() + i * cap;
    char* scratch = buf.data() + TEXT_ILP * cap;
    uint64_t acc = 0;
    for (;;) {
      const size_t b = next.fetch_add(8192);
      if (b >= n) break;
      const size_t e = std::min(n, b + 8192);
      for (size_t k = b; k < e; k += TEXT_ILP) {
        const int m = (int)std::min<size_t>(TEXT_ILP, e - k);
        for (int i = 0; i < m; i++)
          len[i] = orbit ? state_orbit_text_into(L, rows + (k + i) * (size_t)L.W, txt[i], scratch)
                         : state_text_into(L, rows + (k + i) * (size_t)L.W, txt[i], scratch);
        acc += fnv1a64_sum(txt, len, m);
      }
    }
    part[(size_t)t] = acc;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; t++) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  uint64_t sum = 0;
  for (uint64_t v : part) sum += v;
  return sum;
}

extern "C" int rtla_rows_text_hash(const rtla_cfg* c, const uint32_t* rows, size_t n, int threads, uint64_t* out) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!out || (n && !rows)) return RTLA_E_ARG;
  *out = rows_digest(L, rows, n, text_threads(threads));
  return RTLA_OK;
}

extern "C" int rtla_rows_orbit_hash(const rtla_cfg* c, const uint32_t* rows, size_t n, int threads, uint64_t* out) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!out || (n && !rows)) return RTLA_E_ARG;
  *out = rows_digest(L, rows, n, text_threads(threads), true);
  return RTLA_OK;
}

extern "C" int rtla_orbit_text(const rtla_cfg* c, const uint32_t* row, char* buf, size_t cap) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  const size_t tc = state_text_cap(L);
  std::vector<char> b(2 * tc);
  const size_t n = state_orbit_text_into(L, row, b.data(), b.data() + tc);
  if (n + 1 > cap) return RTLA_E_ARG;
  memcpy(buf, b.data(), n);
  buf[n] = 0;
  return (int)n;
}

static int flags_to_status(int flags) {
  if (flags & FLAG_LOCAL_FAILURE) return RTLA_E_HIP;
  if (flags & FLAG_SPEC_ERROR) return RTLA_E_SPEC;
  if (flags) return RTLA_E_OVERFLOW;
  return RTLA_OK;
}

static void report_flags(int flags) {
  if (flags & FLAG_SPEC_ERROR) fprintf(stderr, "rtla: TLC evaluation error in Next (sequence index outside DOMAIN)\n");
  if (flags & FLAG_ROW_OVERFLOW) fprintf(stderr, "rtla: row capacity exceeded (raise bag_cap / elec_cap)\n");
  if (flags & FLAG_FRONTIER_FULL) fprintf(stderr, "rtla: next-frontier buffer full (raise frontier_cap / mem_budget)\n");
  if (flags & FLAG_FPSET_FULL) fprintf(stderr, "rtla: fingerprint set too full (raise fpset_log2)\n");
  if (flags & FLAG_OUTBOX_FULL) fprintf(stderr, "rtla: exchange outbox overflow list full\n");
  if (flags & FLAG_BAD_INDEX) fprintf(stderr, "rtla: checked build: a kernel index left its buffer\n");
  if (flags & FLAG_LOCAL_FAILURE) fprintf(stderr, "rtla: a rank's local work failed\n");
}

// RTLA_XFLAGS: kernel-variant switches (XF_* in rtla_device.h) for performance
// experiments; results are identical for the variants that do not skip work.
static int env_xflags() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTLA_XFLAGS");
    v = e ? (atoi(e) & (XF_GENERIC_DELTA | XF_BLOCK4 | XF_NO_PERSIST | XF_CAS_ONLY | XF_WAVE_KERNEL | XF_NO_SPECIAL)) : 0;
  }
  return v;
}

// Every enabled successor of n device rows (d_rows holds round64(n) rows),
// copied to the host sorted by (input, instance).  The level kernel itself
// runs it -- k_expand_compact with XF_ALL_SUCCESSORS: the same evaluation,
// fingerprint derivation and row building as the BFS, minus the seen set --
// so this parity seam checks the hot kernel; layouts too wide for its LDS
// tile (and RTLA_XFLAGS=2048) use the wave-per-state k_expand_batch.
static int expand_batch_dev(const Layout& L, const uint32_t* d_rows, size_t n, std::vector<uint32_t>& out,
                            std::vector<uint64_t>& info, hipStream_t st) {
  size_t cap = round64(std::max<size_t>(n, 1) * (size_t)L.fam[F_COUNT]);
  uint32_t* d_out = nullptr;
  uint64_t* d_info = nullptr;
  DevCounters* d_ctr = nullptr;
  HIPCHK(hipMalloc(&d_out, cap * L.W * 4));
  HIPCHK(hipMalloc(&d_info, cap * 8));
  HIPCHK(hipMalloc(&d_ctr, sizeof(DevCounters)));
  HIPCHK(hipMemsetAsync(d_ctr, 0, sizeof(DevCounters), st));
  const bool hot = expand_compact_wpb(L) > 0 && !(env_xflags() & XF_WAVE_KERNEL);
  if (hot) {
    const uint64_t caps[3] = {round64(n), cap, cap};  // DevCounters cap_cur / cap_next / cap_parents
    HIPCHK(hipMemcpyAsync(&d_ctr->cap_cur, caps, sizeof caps, hipMemcpyHostToDevice, st));
    const Ring cur{const_cast<uint32_t*>(d_rows), 0, round64(n)}, next{d_out, 0, cap};
    ShardBox box{1, 0, 0, 0, nullptr, nullptr, nullptr};
    HIPCHK(launch_expand(L, cur, 0, n, 0, next, d_info, 0, cap, nullptr, 1, d_ctr, box, 0, st,
                         XF_ALL_SUCCESSORS | XF_NO_COVER, nullptr));
  } else {
    HIPCHK(launch_expand_batch(L, d_rows, n, d_out, d_info, cap, d_ctr, st));
  }
  DevCounters h;
  HIPCHK(hipMemcpyAsync(&h, d_ctr, sizeof h, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  int rc = RTLA_OK;
  if (h.flags) { report_flags(h.flags); rc = flags_to_status(h.flags); }
  size_t m = (size_t)h.next_count;
  out.resize(m * L.W);
  info.resize(m);
  if (m) {
    HIPCHK(hipMemcpy(out.data(), d_out, m * L.W * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(info.data(), d_info, m * 8, hipMemcpyDeviceToHost));
  }
  (void)hipFree(d_out);
  (void)hipFree(d_info);
  (void)hipFree(d_ctr);
  std::vector<size_t> ord(m);
  for (size_t k = 0; k < m; k++) ord[k] = k;
  std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
    uint64_t ka = (info[a] >> 32) << 16 | (info[a] & 0xffff), kb = (info[b] >> 32) << 16 | (info[b] & 0xffff);
    return ka < kb;
  });
  std::vector<uint32_t> o2(m * L.W);
  std::vector<uint64_t> i2(m);
  for (size_t k = 0; k < m; k++) {
    memcpy(&o2[k * L.W], &out[ord[k] * L.W], L.W * 4);
    i2[k] = info[ord[k]];
  }
  out.swap(o2);
  info.swap(i2);
  return rc;
}

extern "C" int rtla_expand_batch(const rtla_cfg* c, const uint32_t* rows, size_t n, uint32_t* succ, uint64_t* info,
                                 size_t cap, size_t* n_out) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!rows || !n_out) return RTLA_E_ARG;
  uint32_t* d_rows = nullptr;
  HIPCHK(hipMalloc(&d_rows, round64(std::max<size_t>(n, 1)) * L.W * 4));
  HIPCHK(hipMemcpy(d_rows, rows, n * L.W * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> out;
  std::vector<uint64_t> inf;
  r = expand_batch_dev(L, d_rows, n, out, inf, nullptr);
  (void)hipFree(d_rows);
  if (r < 0) return r;
  *n_out = inf.size();
  if (inf.size() > cap) return RTLA_E_ARG;
  if (succ) memcpy(succ, out.data(), out.size() * 4);
  if (info) memcpy(info, inf.data(), inf.size() * 8);
  return RTLA_OK;
}

extern "C" int rtla_random_rows(const rtla_cfg* c, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool,
                                uint32_t* rows) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!rows && n) return RTLA_E_ARG;
  for (uint64_t k = 0; k < n; k++) random_state(L, seed, synth_state_id(seed, first + k, pool), rows + k * L.W);
  return RTLA_OK;
}

extern "C" int rtla_random_texts(const rtla_cfg* c, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool,
                                 char* buf, size_t cap, size_t* len) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!len || (!buf && cap)) return RTLA_E_ARG;
  // host threads, each rendering a contiguous slice of the inputs
  const int nt = (int)std::min<uint64_t>(std::max<uint64_t>(n / 256, 1), (uint64_t)text_threads(0));
  std::vector<std::string> part((size_t)nt);
  auto work = [&](int t) {
    const size_t tc = state_text_cap(L);
    std::vector<uint32_t> row(L.W);
    std::vector<char> tmp(2 * tc);
    const uint64_t b = n * t / nt, e = n * (t + 1) / nt;
    std::string& out = part[(size_t)t];
    for (uint64_t k = b; k < e; k++) {
      random_state(L, seed, synth_state_id(seed, first + k, pool), row.data());
      const size_t m = state_text_into(L, row.data(), tmp.data(), tmp.data() + tc);
      out.append(tmp.data(), m);
      out.push_back('\x1e');
    }
  };
  std::vector<std::thread> pool_th;
  for (int t = 1; t < nt; t++) pool_th.emplace_back(work, t);
  work(0);
  for (auto& th : pool_th) th.join();
  size_t at = 0;
  for (auto& p : part) {
    if (at + p.size() <= cap) memcpy(buf + at, p.data(), p.size());
    at += p.size();
  }
  *len = at;
  return at <= cap ? RTLA_OK : RTLA_E_ARG;
}

extern "C" int rtla_comm_id(void* out128) {
  if (!out128) return RTLA_E_ARG;
  const char* tr = getenv("RTLA_TRANSPORT");
  if (tr && !strcmp(tr, "shm")) {  // the id only names the shared-memory segment
    uint64_t v[16];
    const uint64_t t = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    for (int i = 0; i < 16; i++) v[i] = t * 0x9E3779B97F4A7C15ull + (uint64_t)getpid() * 0xBF58476D1CE4E5B9ull + i;
    memcpy(out128, v, 128);
    return RTLA_OK;
  }
  ncclUniqueId id;
  ncclResult_t r0;
  {
    StdoutToStderr quiet;
    r0 = ncclGetUniqueId(&id);
  }
  NCCLCHK(r0);
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  memcpy(out128, &id, 128);
  return RTLA_OK;
}

static void free_shard(Shard& s) {
  void* ptrs[] = {s.table,    s.sent,     s.parents,  s.arena,    s.ctr,       s.dflags,    s.out_count,
                  s.in_count, s.all_count, s.send_fp, s.send_ref, s.send_ans,  s.recv_fp,   s.recv_ans,
                  s.rows_in,  s.rows_base, s.send_rows, s.recv_rows, s.over_fp[0], s.over_fp[1],
                  s.over_ref[0], s.over_ref[1], s.over_cnt};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s.ev0) (void)hipEventDestroy(s.ev0);
  if (s.ev1) (void)hipEventDestroy(s.ev1);
  if (s.evm) (void)hipEventDestroy(s.evm);
  s = Shard();
}

extern "C" void rtla_close(rtla_ctx* x) {
  if (!x) return;
  (void)hipSetDevice(x->device);
  for (auto& s : x->sh) free_shard(s);
  if (x->red) (void)hipFree(x->red);
  if (x->comm) ncclCommDestroy(x->comm);
  if (x->shm) {
    munmap(x->shm->hdr, x->shm->size);
    delete x->shm;
  }
  if (x->stream) (void)hipStreamDestroy(x->stream);
  delete x;
}

static int alloc_shard(rtla_ctx* x, Shard& s, uint64_t budget) {
  const Layout& L = x->L;
  const int G = x->nshard;
  uint64_t tbytes = 8ull << x->tlog2;
  // load factor <= 0.75 (RTLA_MODE_DEDUP: no BFS, no parent records)
  s.parents_cap = x->cfg.mode == RTLA_MODE_DEDUP ? 64 : (1ull << x->tlog2) - (1ull << x->tlog2) / 4;
  uint64_t pbytes = s.parents_cap * 8;
  uint64_t rowb = (uint64_t)L.W * 4;
  uint64_t boxb = G > 1 ? (uint64_t)G * x->box_cap * (16 + 8 + 4 + 16 + 4) +
                              2ull * G * x->rows_cap * (L.W + 2) * 4 + 2ull * x->over_cap * 24
                        : 0;
  const uint64_t sbytes = G > 1 && x->slog2 ? 8ull << x->slog2 : 0;
  if (!x->front_cap) {
    uint64_t used = tbytes + sbytes + pbytes + boxb;
    uint64_t rest = budget > used ? budget - used : 0;
    x->front_cap = std::max<uint64_t>(rest / rowb, 2048);
  }
  x->front_cap = std::max<uint64_t>(x->front_cap & ~63ull, 128);  // whole 64-row groups (Ring)
  HIPCHK(hipMalloc(&s.table, tbytes));
  HIPCHK(hipMalloc(&s.parents, pbytes));
  HIPCHK(hipMalloc(&s.arena, x->front_cap * rowb));
  HIPCHK(hipMalloc(&s.ctr, sizeof(DevCounters)));
  HIPCHK(hipMalloc(&s.dflags, sizeof(int) * 64));
  if (G > 1) {
    HIPCHK(hipMalloc(&s.out_count, 8 * (G + 2)));
    HIPCHK(hipMalloc(&s.in_count, 8 * G));
    HIPCHK(hipMalloc(&s.all_count, 8 * G * (G + 2)));
    HIPCHK(hipMalloc(&s.send_fp, 16 * G * x->box_cap));
    HIPCHK(hipMalloc(&s.send_ref, 8 * G * x->box_cap));
    HIPCHK(hipMalloc(&s.send_ans, 4 * G * x->box_cap));
    HIPCHK(hipMalloc(&s.recv_fp, 16 * G * x->box_cap));
    HIPCHK(hipMalloc(&s.recv_ans, 4 * G * x->box_cap));
    HIPCHK(hipMalloc(&s.rows_in, 8 * G));
    HIPCHK(hipMalloc(&s.rows_base, 8 * G));
    HIPCHK(hipMalloc(&s.send_rows, 4ull * G * x->rows_cap * (L.W + 2)));
    HIPCHK(hipMalloc(&s.recv_rows, 4ull * G * x->rows_cap * (L.W + 2)));
    for (int k = 0; k < 2; k++) {
      HIPCHK(hipMalloc(&s.over_fp[k], 16 * std::max<uint64_t>(x->over_cap, 1)));
      HIPCHK(hipMalloc(&s.over_ref[k], 8 * std::max<uint64_t>(x->over_cap, 1)));
    }
    HIPCHK(hipMalloc(&s.over_cnt, 16));
    HIPCHK(hipMemsetAsync(s.over_cnt, 0, 16, x->stream));
    s.h_out.assign(G + 2, 0);
    s.h_in.assign(G, 0);
    s.h_all.assign((size_t)G * (G + 2), 0);
    if (sbytes) {
      HIPCHK(hipMalloc(&s.sent, sbytes));
      HIPCHK(hipMemsetAsync(s.sent, 0, sbytes, x->stream));
    }
  }
  HIPCHK(hipMemsetAsync(s.table, 0, tbytes, x->stream));
  HIPCHK(hipMemsetAsync(s.ctr, 0, sizeof(DevCounters), x->stream));
  HIPCHK(hipEventCreate(&s.ev0));
  HIPCHK(hipEventCreate(&s.ev1));
  HIPCHK(hipEventCreate(&s.evm));
  return RTLA_OK;
}

// RTLA_FAULT=<where>:<rank> (tests): this rank's local work at <where> fails,
// so the tests can check that the failure reaches every rank promptly.
static bool fault_here(const rtla_ctx* x, const char* where) {
  const char* e = getenv("RTLA_FAULT");
  if (!e) return false;
  const char* colon = strchr(e, ':');
  if (!colon || (size_t)(colon - e) != strlen(where) || strncmp(e, where, colon - e) != 0) return false;
  return atoi(colon + 1) == x->rank;
}

// Sum (op 0) or max (op 1) of n u64 over all ranks; host in/out.
static int allreduce_u64(rtla_ctx* x, uint64_t* v, int n, int op);

// Multi-shard exchange sizing.  Per owner, an outbox region
// of box_cap records (48 B each with the answers and the receiving side):
// ~1/12 of the budget over the G regions.  The level kernel takes frontier
// groups while every region is below stop_at; the groups in flight when one
// fills -- at most one per resident wave, each of whose GROUP states may
// queue every action instance -- spill onto the overflow list (over_cap).
// Without the group queue (the wave-per-state kernel) a round is bounded
// instead, so that no region can overflow (chunk).  Every rank must agree on
// these (round counts and message sizes follow from them): world > 1 takes
// the smallest of each over the ranks.
static int size_exchange(rtla_ctx* x, uint64_t per) {
  const Layout& L = x->L;
  const int G = x->nshard;
  const uint64_t ninst = (uint64_t)L.fam[F_COUNT];  // records one frontier state queues at most
  int waves = 0, group = 0;
  x->guarded = level_kernel_shape(L, true, env_xflags(), &waves, &group);
  x->box_cap = std::max<uint64_t>(per / 12 / ((uint64_t)G * 48), 16 * OBOX_CHUNK);
  if (const char* e = getenv("RTLA_OUTBOX_CAP"))  // tests: tiny regions, many rounds, the overflow list in use
    if (atoll(e) > 0) x->box_cap = std::max<uint64_t>((uint64_t)atoll(e), 16 * OBOX_CHUNK);
  if (x->cfg.chunk) x->chunk = round64(x->cfg.chunk);  // explicit bound on the states a round expands
  else x->chunk = x->guarded ? 0 : std::max<uint64_t>(64, (x->box_cap / ninst) & ~63ull);
  x->over_cap = x->guarded ? (uint64_t)waves * (uint64_t)group * ninst : 0;
  // the two overflow lists (24 B a record) take at most 1/16 of the budget: a
  // small budget bounds the states a round expands instead, so that even
  // then every record of a launch would fit the list
  const uint64_t over_room = std::max<uint64_t>(per / 16 / 48, 64 * ninst);
  if (x->over_cap > over_room) {
    x->over_cap = over_room;
    const uint64_t c = std::max<uint64_t>(64, (over_room / ninst) & ~63ull);
    x->chunk = x->chunk ? std::min(x->chunk, c) : c;
  }
  // re-balancing staging: ~1/20 of the budget; more rows move in sub-rounds
  x->rows_cap = (per / 20) / (2ull * G * (L.W + 2) * 4);
  x->rows_cap = std::min<uint64_t>(std::max<uint64_t>(x->rows_cap, 256), x->box_cap);
  if (const char* e = getenv("RTLA_ROWS_CAP"))  // tests: tiny staging, every re-balancing move in sub-rounds
    if (atoll(e) > 0) x->rows_cap = std::min<uint64_t>((uint64_t)atoll(e), x->box_cap);
  if (x->world > 1) {  // min over the ranks (max of the complements); the overflow bound: max
    uint64_t v[5] = {~x->box_cap, ~(x->chunk ? x->chunk : ~0ull), ~x->rows_cap, x->over_cap, x->guarded ? 0ull : 1ull};
    if (int rc = allreduce_u64(x, v, 5, 1)) return rc;
    x->box_cap = ~v[0];
    x->chunk = ~v[1] == ~0ull ? 0 : ~v[1];
    x->rows_cap = ~v[2];
    x->over_cap = v[3];
    if (v[4] && x->guarded) {  // some rank runs the wave-per-state kernel: all bound their rounds alike
      x->guarded = false;
      if (!x->chunk) x->chunk = std::max<uint64_t>(64, (x->box_cap / ninst) & ~63ull);
    }
  }
  x->stop_at = x->box_cap - std::max<uint64_t>(x->box_cap / 8, OBOX_CHUNK);
  return RTLA_OK;
}

extern "C" int rtla_open(const rtla_cfg* cfg, int rank, int world, const void* comm_id, rtla_ctx** out) {
  if (!cfg || !out || world < 1 || rank < 0 || rank >= world) return RTLA_E_ARG;
  *out = nullptr;
  if (world > 1 && !comm_id) return RTLA_E_ARG;
  if (world > 1 && cfg->shards > 1) return RTLA_E_CONFIG;
  if (world > SHARD_MAX || cfg->shards > SHARD_MAX) return RTLA_E_CONFIG;  // per-owner outbox state is sized by it
  if (cfg->mode != RTLA_MODE_BFS && (cfg->mode != RTLA_MODE_DEDUP || world > 1 || cfg->shards > 1))
    return RTLA_E_CONFIG;
  rtla_ctx* x = new rtla_ctx();
  x->cfg = *cfg;
  int r = layout_from_cfg(cfg, &x->L);
  if (r) { delete x; return r; }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) { delete x; return RTLA_E_HIP; }
  x->rank = rank;
  x->world = world;
  x->device = rank % ndev;
  x->nshard = world > 1 ? world : std::max(1, cfg->shards);
  x->shard0 = world > 1 ? rank : 0;
  int nlocal = world > 1 ? 1 : x->nshard;
  if (hipSetDevice(x->device) != hipSuccess) { delete x; return RTLA_E_HIP; }
  if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) { delete x; return RTLA_E_HIP; }
  if (hipMalloc(&x->red, 64 * 8) != hipSuccess) { rtla_close(x); return RTLA_E_HIP; }
  if (world > 1) {
    const char* tr = getenv("RTLA_TRANSPORT");
    if (tr && !strcmp(tr, "shm")) {
      if (shm_open_comm(x, comm_id) != RTLA_OK) { rtla_close(x); return RTLA_E_COMM; }
    } else {
      ncclUniqueId id;
      memcpy(&id, comm_id, sizeof id);
      ncclResult_t r0;
      {
        StdoutToStderr quiet;
        r0 = ncclCommInitRank(&x->comm, world, id, rank);
      }
      if (r0 != ncclSuccess) { rtla_close(x); return RTLA_E_COMM; }
    }
  } else if (x->nshard > 1) {
    const char* tr = getenv("RTLA_TRANSPORT");
    if (tr && !strcmp(tr, "rccl")) {  // virtual shards exchanging through a one-rank RCCL communicator
      ncclUniqueId id;
      ncclResult_t r0;
      {
        StdoutToStderr quiet;
        r0 = ncclGetUniqueId(&id);
        if (r0 == ncclSuccess) r0 = ncclCommInitRank(&x->comm, 1, id, 0);
      }
      if (r0 != ncclSuccess) {
        rtla_close(x);
        return RTLA_E_COMM;
      }
      x->rccl_local = true;
    }
  }
  // From here on (world > 1) every rank reaches the same collectives: a local
  // failure is carried to the last one, which fails every rank together.
  int err = RTLA_OK;
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  uint64_t budget = cfg->mem_budget ? cfg->mem_budget : (uint64_t)(free_b * 0.85);
  uint64_t per = budget / nlocal;
  const Layout& L = x->L;
  const int G = x->nshard;
  if (G > 1)
    if (int rc = size_exchange(x, per)) { rtla_close(x); return rc; }
  int tl = cfg->fpset_log2;
  if (!tl) {
    tl = 20;
    // the fingerprint set (multi-shard: + the sent cache, half its size): ~40% of the budget
    const uint64_t tshare = G > 1 ? per * 4 / 15 : per * 2 / 5;
    while (tl < 34 && (8ull << (tl + 1)) <= tshare) tl++;
  }
  if (tl < 10 || tl > 40) err = RTLA_E_CONFIG;
  x->tlog2 = tl;
  // the sent cache is a dedup hint (one slot per fingerprint, overwritten on
  // a miss): half the set's slots (configs[1], 8 shards: a quarter sends 8 %
  // more records and takes 5 % longer, profiles/r05_v2); RTLA_SENT_CACHE=0
  // turns it off (every remote successor is queued for its owner: 1.34x slower)
  const char* sc = getenv("RTLA_SENT_CACHE");
  x->slog2 = sc && atoi(sc) == 0 ? 0 : std::max(12, tl - 1);
  if (const char* sl = getenv("RTLA_SENT_LOG2"))  // experiments: the sent cache's size (log2 slots)
    if (x->slog2 && atoi(sl) >= 12 && atoi(sl) <= 36) x->slog2 = atoi(sl);
  x->front_cap = cfg->frontier_cap;
  x->sh.resize(nlocal);
  for (int k = 0; k < nlocal && !err; k++) {
    x->sh[k].id = x->shard0 + k;
    if (alloc_shard(x, x->sh[k], per) != RTLA_OK) {
      fprintf(stderr, "rtla: device allocation failed (fpset 2^%d slots, frontier 2x%llu rows of %d B)\n", tl,
              (unsigned long long)x->front_cap, L.W * 4);
      err = RTLA_E_HIP;
    }
  }
  if (!err && (hipStreamSynchronize(x->stream) != hipSuccess || fault_here(x, "open"))) err = RTLA_E_HIP;
  if (world > 1) {  // every rank opened, or none
    uint64_t bad = err ? 1 : 0;
    if (int rc = allreduce_u64(x, &bad, 1, 1)) err = err ? err : rc;
    else if (bad && !err) err = RTLA_E_COMM;
  }
  if (err) {
    rtla_close(x);
    return err;
  }
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, x->device);
  x->grid = prop.multiProcessorCount * expand_blocks_per_cu(L) * 2;
  *out = x;
  return RTLA_OK;
}

extern "C" int rtla_device_info(rtla_ctx* x, char* buf, size_t cap) {
  if (!x || !buf) return RTLA_E_ARG;
  std::string fr;  // this process's shards' current levels
  for (auto& s : x->sh) fr += (fr.empty() ? "" : ", ") + std::to_string(s.n_cur);
  hipDeviceProp_t p;
  HIPCHK(hipGetDeviceProperties(&p, x->device));
  snprintf(buf, cap,
           "{\"device\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"rank\": %d, \"world\": %d, \"shards\": %d, "
           "\"fpset_slots_log2\": %d, \"frontier_cap\": %llu, \"row_words\": %d, \"grid\": %d, \"chunk\": %llu, "
           "\"transport\": \"%s\", \"sent_cache_slots_log2\": %d, \"rebalanced_rows\": %llu, "
           "\"outbox_records_per_owner\": %llu, \"overflow_records\": %llu, \"exchange_rounds\": %llu, "
           "\"overflowed_records\": %llu, \"records_sent\": %llu, \"shard_frontier\": [%s]}",
           p.name, p.gcnArchName, p.multiProcessorCount, x->rank, x->world, x->nshard, x->tlog2,
           (unsigned long long)x->front_cap, x->L.W, x->grid, (unsigned long long)x->chunk,
           x->shm ? "shm" : x->comm ? (x->rccl_local ? "rccl-local" : "rccl") : "device", x->nshard > 1 ? x->slog2 : 0,
           (unsigned long long)x->rebalanced, (unsigned long long)x->box_cap, (unsigned long long)x->over_cap,
           (unsigned long long)x->rounds, (unsigned long long)x->overflowed, (unsigned long long)x->records,
           fr.c_str());
  return RTLA_OK;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Sum of n1 u64 and max of n2 u64 over all ranks (one synchronisation); host in/out.
static int allreduce2_u64(rtla_ctx* x, uint64_t* sum, int n1, uint64_t* mx, int n2) {
  if (x->world == 1 && !x->rccl_local) return RTLA_OK;
  HIPCHK(hipMemcpyAsync(x->red, sum, 8 * n1, hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipMemcpyAsync(x->red + 32, mx, 8 * n2, hipMemcpyHostToDevice, x->stream));
  if (!x->shm) {  // both reductions in one group (closed also when one could not be posted)
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(r, __LINE__);
    r = ncclAllReduce(x->red, x->red, n1, ncclUint64, ncclSum, x->comm, x->stream);
    if (r == ncclSuccess) r = ncclAllReduce(x->red + 32, x->red + 32, n2, ncclUint64, ncclMax, x->comm, x->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) return nccl_fail(r, __LINE__);
  } else {
    if (int rc = comm_allreduce(x, x->red, n1, 0)) return rc;
    if (int rc = comm_allreduce(x, x->red + 32, n2, 1)) return rc;
  }
  HIPCHK(hipMemcpyAsync(sum, x->red, 8 * n1, hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipMemcpyAsync(mx, x->red + 32, 8 * n2, hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  return RTLA_OK;
}

// Sum (op 0) or max (op 1) of n u64 over all ranks; host in/out.
static int allreduce_u64(rtla_ctx* x, uint64_t* v, int n, int op) {
  if (x->world == 1 && !x->rccl_local) return RTLA_OK;
  HIPCHK(hipMemcpyAsync(x->red, v, 8 * n, hipMemcpyHostToDevice, x->stream));
  if (int rc = comm_allreduce(x, x->red, n, op)) return rc;
  HIPCHK(hipMemcpyAsync(v, x->red, 8 * n, hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  return RTLA_OK;
}

// ---- checkpoint / recover (TLC's -checkpoint / -recover and its states/
// directory, reference .gitignore:2).  One file per shard:
// <prefix>.shard<id>.rtla = header | fingerprint set | sent cache (G > 1) |
// parent records [0, cur_base + n_cur) | current frontier rows | coverage.
// Written between levels; a context opened with the same configuration
// (same cfg, fingerprint-set size and shard count) resumes from it.
namespace {
struct CkptHeader {
  char magic[8];
  int32_t abi, nshard, shard, W, tlog2, level;
  rtla_cfg cfg;
  uint64_t distinct, generated, max_front, cur_base, n_cur, parents_n;
  int32_t finished, viol_mask, viol_in_model, viol_inst;
  uint64_t viol_parent, viol_child;
};

bool write_all(FILE* f, const void* p, size_t n) { return fwrite(p, 1, n, f) == n; }
bool read_all(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

// device <-> file through a bounded host staging buffer
bool dev_to_file(FILE* f, const void* d, size_t n, std::vector<char>& buf) {
  for (size_t off = 0; off < n; off += buf.size()) {
    const size_t m = std::min(buf.size(), n - off);
    if (hipMemcpy(buf.data(), (const char*)d + off, m, hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (!write_all(f, buf.data(), m)) return false;
  }
  return true;
}
bool file_to_dev(FILE* f, void* d, size_t n, std::vector<char>& buf) {
  for (size_t off = 0; off < n; off += buf.size()) {
    const size_t m = std::min(buf.size(), n - off);
    if (!read_all(f, buf.data(), m)) return false;
    if (hipMemcpy((char*)d + off, buf.data(), m, hipMemcpyHostToDevice) != hipSuccess) return false;
  }
  return true;
}
bool ring_to_file(FILE* f, const Ring& r, int W, uint64_t n, std::vector<char>& buf) {
  for (uint64_t g = 0; g < n;) {
    const uint64_t p = ring_idx(r, g), m = std::min<uint64_t>(n - g, r.cap - p);
    if (!dev_to_file(f, r.base + p * (uint64_t)W, m * W * 4, buf)) return false;
    g += m;
  }
  return true;
}
std::string ckpt_path(const char* prefix, int shard) {
  return std::string(prefix) + ".shard" + std::to_string(shard) + ".rtla";
}
}  // namespace

// Collective when world > 1: every rank reaches every reduction below, also
// after a local failure (its flag travels in the reduction), so one rank's
// error is every rank's error and no rank is left waiting in a collective.
extern "C" int rtla_checkpoint(rtla_ctx* x, const char* prefix) {
  if (!x || !prefix) return RTLA_E_ARG;
  if (!x->inited) return RTLA_E_STATE;
  std::vector<char> buf(64 << 20);
  // Each shard is written to <path>.tmp (flushed to disk); only when every
  // shard of every rank has been written are the files renamed over the
  // previous checkpoint, so a crash mid-write leaves the last good one intact.
  uint64_t failed = hipSetDevice(x->device) != hipSuccess || hipStreamSynchronize(x->stream) != hipSuccess ? 1 : 0;
  for (auto& s : x->sh) {
    if (failed) break;
    CkptHeader h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, "RTLACKP1", 8);
    h.abi = RTLA_ABI_VERSION; h.nshard = x->nshard; h.shard = s.id; h.W = x->L.W; h.tlog2 = x->tlog2;
    h.level = x->level; h.cfg = x->cfg;
    h.distinct = x->distinct; h.generated = x->generated; h.max_front = x->max_front;
    h.cur_base = s.cur_base; h.n_cur = s.n_cur; h.parents_n = s.cur_base + s.n_cur;
    h.finished = x->finished; h.viol_mask = s.viol_mask; h.viol_in_model = s.viol_in_model;
    h.viol_inst = s.viol_inst; h.viol_parent = s.viol_parent; h.viol_child = s.viol_child;
    const std::string tmp = ckpt_path(prefix, s.id) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) { failed = 1; break; }
    DevCounters c;
    bool ok = write_all(f, &h, sizeof h) && dev_to_file(f, s.table, 8ull << x->tlog2, buf) &&
              (!s.sent || dev_to_file(f, s.sent, 8ull << x->slog2, buf)) &&
              dev_to_file(f, s.parents, 8 * h.parents_n, buf) &&
              ring_to_file(f, cur_ring(x, s), x->L.W, s.n_cur, buf) &&
              hipMemcpy(&c, s.ctr, sizeof c, hipMemcpyDeviceToHost) == hipSuccess &&
              write_all(f, c.cover, sizeof c.cover);
    ok = ok && fflush(f) == 0 && fsync(fileno(f)) == 0;
    ok = fclose(f) == 0 && ok;
    if (!ok) { failed = 1; break; }
  }
  if (int rc = allreduce_u64(x, &failed, 1, 1)) return rc;
  if (failed) {
    for (auto& s : x->sh) (void)remove((ckpt_path(prefix, s.id) + ".tmp").c_str());
    return RTLA_E_ARG;
  }
  // the renames are agreed on too: every rank reports the same outcome
  uint64_t renamed_bad = 0;
  for (auto& s : x->sh) {
    const std::string path = ckpt_path(prefix, s.id);
    if (rename((path + ".tmp").c_str(), path.c_str()) != 0) renamed_bad = 1;
  }
  if (int rc = allreduce_u64(x, &renamed_bad, 1, 1)) return rc;
  if (renamed_bad) {
    fprintf(stderr, "rtla: checkpoint %s: a shard file could not be renamed into place "
                    "(the checkpoint mixes generations; recover will refuse it)\n", prefix);
    return RTLA_E_ARG;
  }
  return RTLA_OK;
}

extern "C" int rtla_recover(rtla_ctx* x, const char* prefix) {
  if (!x || !prefix) return RTLA_E_ARG;
  if (x->cfg.mode == RTLA_MODE_DEDUP) return RTLA_E_STATE;
  std::vector<char> buf(64 << 20);
  int level = -1;
  int err = hipSetDevice(x->device) != hipSuccess ? RTLA_E_HIP : RTLA_OK;  // the first local failure
  for (auto& s : x->sh) {
    if (err) break;
    FILE* f = fopen(ckpt_path(prefix, s.id).c_str(), "rb");
    if (!f) { err = RTLA_E_ARG; break; }
    CkptHeader h;
    bool ok = read_all(f, &h, sizeof h) && memcmp(h.magic, "RTLACKP1", 8) == 0 && h.abi == RTLA_ABI_VERSION &&
              h.nshard == x->nshard && h.shard == s.id && h.W == x->L.W && h.tlog2 == x->tlog2 &&
              memcmp(&h.cfg, &x->cfg, offsetof(rtla_cfg, fpset_log2)) == 0 && h.parents_n <= s.parents_cap &&
              h.n_cur <= x->front_cap && (level < 0 || level == h.level);
    DevCounters c;
    memset(&c, 0, sizeof c);
    ok = ok && file_to_dev(f, s.table, 8ull << x->tlog2, buf) &&
         (!s.sent || file_to_dev(f, s.sent, 8ull << x->slog2, buf)) &&
         file_to_dev(f, s.parents, 8 * h.parents_n, buf) &&
         file_to_dev(f, s.arena, 4ull * x->L.W * h.n_cur, buf) && read_all(f, c.cover, sizeof c.cover);
    fclose(f);
    if (!ok) { err = RTLA_E_STATE; break; }
    if (hipMemcpy(s.ctr, &c, sizeof c, hipMemcpyHostToDevice) != hipSuccess) { err = RTLA_E_HIP; break; }
    level = h.level;
    s.cur_start = 0; s.cur_base = h.cur_base; s.n_cur = h.n_cur;
    s.viol_mask = h.viol_mask; s.viol_in_model = h.viol_in_model; s.viol_inst = h.viol_inst;
    s.viol_parent = h.viol_parent; s.viol_child = h.viol_child;
    x->level = h.level; x->distinct = h.distinct; x->generated = h.generated; x->max_front = h.max_front;
    x->finished = h.finished != 0;
  }
  if (x->world > 1) {  // every rank must resume from the same level of the same search
    uint64_t v[7] = {(uint64_t)x->level, x->distinct, x->generated, ~(uint64_t)x->level, ~x->distinct, ~x->generated,
                     err ? 1ull : 0ull};
    if (int rc = allreduce_u64(x, v, 7, 1)) return rc;
    if (err) return err;
    if (v[6]) {
      fprintf(stderr, "rtla: recover failed on another rank\n");
      return RTLA_E_STATE;
    }
    if (v[0] != ~v[3] || v[1] != ~v[4] || v[2] != ~v[5]) {
      fprintf(stderr, "rtla: checkpoint files of different ranks are from different levels\n");
      return RTLA_E_STATE;
    }
  } else if (err) {
    return err;
  }
  x->init_row.assign(x->L.W, 0);
  row_init(x->L, x->init_row.data());
  x->inited = true;
  return RTLA_OK;
}

extern "C" int rtla_reset(rtla_ctx* x) {
  if (!x) return RTLA_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  for (auto& s : x->sh) {
    HIPCHK(hipMemsetAsync(s.table, 0, 8ull << x->tlog2, x->stream));
    if (s.sent) HIPCHK(hipMemsetAsync(s.sent, 0, 8ull << x->slog2, x->stream));
    HIPCHK(hipMemsetAsync(s.ctr, 0, sizeof(DevCounters), x->stream));
    s.n_cur = 0; s.cur_base = 0; s.cur_start = 0;
    s.viol_mask = 0; s.viol_in_model = 0; s.viol_inst = -1; s.viol_parent = 0; s.viol_child = ~0ull;
  }
  HIPCHK(hipStreamSynchronize(x->stream));
  x->inited = false; x->finished = false; x->level = 0; x->distinct = 0; x->generated = 0; x->max_front = 0;
  return RTLA_OK;
}

extern "C" int rtla_init(rtla_ctx* x, rtla_level_stats* st) {
  if (!x) return RTLA_E_ARG;
  if (x->inited || x->cfg.mode == RTLA_MODE_DEDUP) return RTLA_E_STATE;
  double t0 = now_s();
  HIPCHK(hipSetDevice(x->device));
  const Layout& L = x->L;
  x->init_row.assign(L.W, 0);
  row_init(L, x->init_row.data());
  // Init belongs to the shard that owns its fingerprint (raft.tla:155-160: one state)
  int owner = fp_owner(row_fp(x->init_row.data()), x->nshard);
  for (auto& s : x->sh) {
    s.cur_start = 0; s.cur_base = 0; s.n_cur = 0;
    if (s.id != owner) continue;
    HIPCHK(hipMemcpyAsync(s.arena, x->init_row.data(), L.W * 4, hipMemcpyHostToDevice, x->stream));
    HIPCHK(launch_insert_rows(L, s.arena, 1, s.table, x->tlog2, s.dflags, s.ctr, x->stream));
    uint64_t root = ~0ull;
    HIPCHK(hipMemcpyAsync(s.parents, &root, 8, hipMemcpyHostToDevice, x->stream));
    s.n_cur = 1;
  }
  HIPCHK(hipStreamSynchronize(x->stream));
  x->level = 1; x->distinct = 1; x->generated = 1; x->inited = true; x->max_front = 1;
  int bad = check_invariants<0>(L, x->init_row.data(), (const Delta*)nullptr);
  int status = RTLA_OK;
  if (bad) {
    for (auto& s : x->sh)
      if (s.id == owner) { s.viol_mask = bad; s.viol_in_model = 1; s.viol_child = 0; s.viol_inst = -1; }
    x->finished = true;
    status = RTLA_VIOLATION;
  }
  if (st) {
    memset(st, 0, sizeof *st);
    st->level = 1; st->status = status; st->new_states = 1; st->generated = 1;
    st->distinct_total = 1; st->generated_total = 1; st->seconds = now_s() - t0;
    st->row_bytes = (uint64_t)L.W * 4;
  }
  return status;
}

// ---- multi-shard exchange (transport: device copies for local shards, RCCL across ranks)
//
// Two-phase: only fingerprints and answers cross shards.
// One exchange round: the level kernel queues (fingerprint, parent) records
// of successors other shards own; ONE host synchronisation learns every
// (sender, owner) record count, which sizes the fingerprint transfer and the
// answers coming back; the owners insert and answer new / seen; each sender
// builds its winners into its own next level (k_build_winners).  At the
// level's end the shards' next levels are re-balanced (rebalance) -- the only
// rows that ever move, and only what drifted from an even split.

// One exchange between the shards of this process: device copies, or (rccl_local)
// one RCCL group of ncclSend/ncclRecv pairs to rank 0 -- this process -- issued
// in the same order, so the i-th send feeds the i-th receive.
struct Local {
  rtla_ctx* x;
  std::vector<Msg> sends, recvs;
  explicit Local(rtla_ctx* x_) : x(x_) {}
  int move(void* dst, const void* src, size_t bytes) {
    if (!x->rccl_local) {
      HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, x->stream));
      return RTLA_OK;
    }
    sends.push_back({const_cast<void*>(src), bytes, 0});
    recvs.push_back({dst, bytes, 0});
    return RTLA_OK;
  }
  int flush() { return sends.empty() ? RTLA_OK : comm_exchange(x, sends, recvs); }
};

// (1) The round's one synchronisation: every shard's out_count row (records
// reserved per owner, frontier states left, overflow records) -> x->h_rows
// on every rank; h_out[p] = records this shard sends owner p, h_in[p] =
// records it receives from p (reservations past a region's end are on the
// overflow list: counted up to box_cap); in_count on the device.
static int gather_counts(rtla_ctx* x) {
  const int G = x->nshard, RW = G + 2;
  x->h_rows.assign((size_t)G * RW, 0);
  if (x->world == 1) {
    for (auto& s : x->sh) {
      if (x->rccl_local) {  // (one rank: all_count[0, RW) = out_count)
        if (int rc = comm_allgather(x, s.out_count, s.all_count, RW)) return rc;
        HIPCHK(hipMemcpyAsync(x->h_rows.data() + (size_t)s.id * RW, s.all_count, 8 * RW, hipMemcpyDeviceToHost,
                              x->stream));
      } else {
        HIPCHK(hipMemcpyAsync(x->h_rows.data() + (size_t)s.id * RW, s.out_count, 8 * RW, hipMemcpyDeviceToHost,
                              x->stream));
      }
    }
    HIPCHK(hipStreamSynchronize(x->stream));
  } else {
    Shard& s = x->sh[0];
    if (int rc = comm_allgather(x, s.out_count, s.all_count, RW)) return rc;
    HIPCHK(hipMemcpyAsync(x->h_rows.data(), s.all_count, 8 * G * RW, hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipStreamSynchronize(x->stream));
  }
  for (auto& s : x->sh)
    for (int p = 0; p < G; p++) {
      s.h_out[p] = std::min(x->h_rows[(size_t)s.id * RW + p], x->box_cap);
      s.h_in[p] = std::min(x->h_rows[(size_t)p * RW + s.id], x->box_cap);
    }
  // h_in stays untouched until the next round's synchronisation
  for (auto& s : x->sh) HIPCHK(hipMemcpyAsync(s.in_count, s.h_in.data(), 8 * G, hipMemcpyHostToDevice, x->stream));
  return RTLA_OK;
}

// Move the queued (fingerprint) records to their owners.
static int move_fps(rtla_ctx* x) {
  const int G = x->nshard;
  const uint64_t cap = x->box_cap;
  if (x->world == 1) {
    Local lc(x);
    for (auto& dst : x->sh)
      for (auto& src : x->sh) {
        const uint64_t n = src.h_out[dst.id];
        if (n)
          if (int rc = lc.move(dst.recv_fp + 2 * (uint64_t)src.id * cap, src.send_fp + 2 * (uint64_t)dst.id * cap,
                               16 * n))
            return rc;
      }
    return lc.flush();
  }
  Shard& s = x->sh[0];
  std::vector<Msg> sends, recvs;
  for (int p = 0; p < G; p++) {
    if (p == s.id) continue;
    if (s.h_out[p]) sends.push_back({s.send_fp + 2 * (uint64_t)p * cap, 16 * s.h_out[p], p});
    if (s.h_in[p]) recvs.push_back({s.recv_fp + 2 * (uint64_t)p * cap, 16 * s.h_in[p], p});
  }
  return comm_exchange(x, sends, recvs);
}

// (2) Owners answered in recv_ans (0 = seen, nonzero = new): route the
// answers back into the senders' send_ans (sizes known since gather_counts:
// no synchronisation).
static int move_answers(rtla_ctx* x) {
  const int G = x->nshard;
  const uint64_t cap = x->box_cap;
  if (x->world == 1) {
    Local lc(x);
    for (auto& src : x->sh)
      for (auto& dst : x->sh) {
        const uint64_t n = src.h_out[dst.id];
        if (n)
          if (int rc = lc.move(src.send_ans + (uint64_t)dst.id * cap, dst.recv_ans + (uint64_t)src.id * cap, 4 * n))
            return rc;
      }
    return lc.flush();
  }
  Shard& s = x->sh[0];
  std::vector<Msg> sends, recvs;
  for (int p = 0; p < G; p++) {
    if (p == s.id) continue;
    if (s.h_in[p]) sends.push_back({s.recv_ans + (uint64_t)p * cap, 4 * s.h_in[p], p});
    if (s.h_out[p]) recvs.push_back({s.send_ans + (uint64_t)p * cap, 4 * s.h_out[p], p});
  }
  return comm_exchange(x, sends, recvs);
}

// Level end: even out the shards' next levels.  n[k] = next-level states of
// shard k (global ids, the same on every rank); the split every rank computes
// alike is total / G each (the first total % G shards one more); shards
// above it send their LAST rows, in shard order, to those below it (rows and
// parent records, staged k_stage_rows -> exchange -> k_unpack_rows, in
// sub-rounds of rows_cap).  Skipped while the largest excess is within
// 1 % + 64 rows of the split: a new state is stored by the shard that
// generated it, so an even level stays about even, and after the first
// levels (Init's successors all come from Init's shard) little moves.
static int rebalance(rtla_ctx* x, std::vector<uint64_t>& n, const std::vector<uint64_t>& next_base,
                     const std::vector<uint64_t>& next_cap) {
  const int G = x->nshard;
  uint64_t total = 0;
  for (int k = 0; k < G; k++) total += n[k];
  std::vector<uint64_t> tgt(G);
  uint64_t worst = 0;
  for (int k = 0; k < G; k++) {
    tgt[k] = total / G + ((uint64_t)k < total % G ? 1 : 0);
    if (n[k] > tgt[k]) worst = std::max(worst, n[k] - tgt[k]);
  }
  if (worst <= 64 + total / (100ull * G)) return RTLA_OK;
  auto local = [&](int id) -> Shard* {
    for (auto& s : x->sh)
      if (s.id == id) return &s;
    return nullptr;
  };
  struct Move { int a, b; uint64_t first, base, cnt; };  // a's states [first, +cnt) -> b's slots [base, +cnt)
  std::vector<Move> mv;
  std::vector<uint64_t> m = n;
  for (int a = 0, b = 0;;) {  // greedy, in shard order: the same plan on every rank
    while (a < G && m[a] <= tgt[a]) a++;
    while (b < G && m[b] >= tgt[b]) b++;
    if (a >= G || b >= G) break;
    const uint64_t c = std::min(m[a] - tgt[a], tgt[b] - m[b]);
    mv.push_back({a, b, m[a] - c, m[b], c});
    m[a] -= c;
    m[b] += c;
  }
  // a receiver's room (its arena / parent records, as the level kernel's
  // next_cap) is known only where it lives: if any lacks it, nobody moves
  uint64_t short_of_room = 0;
  for (size_t k = 0; k < x->sh.size(); k++)
    if (m[x->sh[k].id] > next_cap[k]) short_of_room = 1;
  if (x->world > 1)
    if (int rc = allreduce_u64(x, &short_of_room, 1, 1)) return rc;
  if (short_of_room || mv.empty()) return RTLA_OK;
  const uint64_t rc = x->rows_cap, RW = (uint64_t)x->L.W + 2;
  uint64_t most = 0;
  for (auto& t : mv) most = std::max(most, t.cnt);
  for (uint64_t lo = 0; lo < most; lo += rc) {
    for (auto& s : x->sh) std::fill(s.h_reb, s.h_reb + 2 * SHARD_MAX, 0ull);
    std::vector<Msg> sends, recvs;
    Local lc(x);
    uint64_t mx = 0;
    for (auto& t : mv) {
      if (t.cnt <= lo) continue;
      const uint64_t c = std::min(rc, t.cnt - lo);
      mx = std::max(mx, c);
      Shard* sa = local(t.a);
      Shard* sb = local(t.b);
      if (sa) {
        const size_t ka = (size_t)(sa - x->sh.data());
        HIPCHK(launch_stage_rows(x->L.W, next_ring(x, *sa), sa->parents, next_base[ka], t.first + lo, c,
                                 sa->send_rows + (uint64_t)t.b * rc * RW, x->stream));
      }
      if (sb) {
        sb->h_reb[t.a] = c;
        sb->h_reb[SHARD_MAX + t.a] = t.base + lo;
      }
      if (x->world == 1) {
        if (int r = lc.move(sb->recv_rows + (uint64_t)t.a * rc * RW, sa->send_rows + (uint64_t)t.b * rc * RW,
                            4 * c * RW))
          return r;
      } else if (sa) {
        sends.push_back({sa->send_rows + (uint64_t)t.b * rc * RW, 4 * c * RW, t.b});
      } else if (sb) {
        recvs.push_back({sb->recv_rows + (uint64_t)t.a * rc * RW, 4 * c * RW, t.a});
      }
    }
    if (x->world == 1) {
      if (int r = lc.flush()) return r;
    } else if (int r = comm_exchange(x, sends, recvs)) {
      return r;
    }
    for (size_t k = 0; k < x->sh.size(); k++) {
      Shard& s = x->sh[k];
      bool any = false;
      for (int p = 0; p < G; p++) any |= s.h_reb[p] != 0;
      if (!any) continue;
      HIPCHK(hipMemcpyAsync(s.rows_in, s.h_reb, 8 * G, hipMemcpyHostToDevice, x->stream));
      HIPCHK(hipMemcpyAsync(s.rows_base, s.h_reb + SHARD_MAX, 8 * G, hipMemcpyHostToDevice, x->stream));
      HIPCHK(launch_unpack_rows(x->L.W, s.recv_rows, s.rows_in, s.rows_base, G, rc, next_ring(x, s), s.parents,
                                next_base[k], next_cap[k], s.ctr, mx, x->stream));
    }
    HIPCHK(hipStreamSynchronize(x->stream));  // (h_reb is rewritten by the next sub-round)
  }
  for (auto& t : mv) {
    if (local(t.a)) x->rebalanced += t.cnt;
  }
  n = m;
  return RTLA_OK;
}

// RTLA_STAMPS builds with RTLA_STAMPS_PRINT set: where the level kernel's
// wave-cycles went (diagnostic).
static void print_stamps(const DevCounters& c, int level) {
  if (!getenv("RTLA_STAMPS_PRINT")) return;
  if (c.cas) fprintf(stderr, "cas level %d: %llu pipelined CAS, %llu probes, %llu new\n", level,
                     (unsigned long long)c.cas, (unsigned long long)c.probes, (unsigned long long)c.next_count);
  static const char* ph[8] = {"group", "ring", "compute", "resolve", "issue", "rows", "drain", "keys+end"};
  // (non-symmetric kernels: "drain" = the group-end row build, "keys+end" = the group-end probe drain)
  unsigned long long tot = 0;
  for (int k = 0; k < 8; k++) tot += c.stamp[k];
  if (!tot) return;
  fprintf(stderr, "stamps level %d:", level);
  for (int k = 0; k < 8; k++) fprintf(stderr, " %s %.3f", ph[k], (double)c.stamp[k] / tot);
  fprintf(stderr, " (%.3g wave-cycles)\n", (double)tot);
}

extern "C" int rtla_step(rtla_ctx* x, rtla_level_stats* st) {
  if (!x) return RTLA_E_ARG;
  if (!x->inited || x->finished) return RTLA_E_STATE;
  double t0 = now_s();
  HIPCHK(hipSetDevice(x->device));
  const Layout& L = x->L;
  const int G = x->nshard;
  std::vector<uint64_t> next_base(x->sh.size()), next_cap(x->sh.size());
  // capacity shortfalls found here travel in the level's reduction like the kernels' flags
  // (a rank returning before the collectives would leave the others waiting in them)
  int lflags = 0;
  for (size_t k = 0; k < x->sh.size(); k++) {
    Shard& s = x->sh[k];
    HIPCHK(hipMemsetAsync(s.ctr, 0, offsetof(DevCounters, cover), x->stream));
    next_base[k] = s.cur_base + s.n_cur;
    const bool no_room = next_base[k] >= s.parents_cap;
    if (no_room) {  // nothing fits: every new state is flagged, none stored
      lflags |= FLAG_FRONTIER_FULL;
      next_base[k] = s.parents_cap;
    }
    next_cap[k] = no_room ? 0 : std::min<uint64_t>(next_room(x, s), s.parents_cap - next_base[k]);
    s.h_caps[0] = s.n_cur; s.h_caps[1] = next_cap[k]; s.h_caps[2] = s.parents_cap;
    HIPCHK(hipMemcpyAsync(&s.ctr->cap_cur, s.h_caps, sizeof s.h_caps, hipMemcpyHostToDevice, x->stream));
  }
  for (auto& s : x->sh) HIPCHK(hipEventRecord(s.ev0, x->stream));
  if (G == 1) {
    Shard& s = x->sh[0];
    ShardBox box{1, 0, 0, 0, nullptr, nullptr, nullptr};
    uint64_t blocks = (s.n_cur + 3) / 4;
    int grid = (int)std::min<uint64_t>(blocks, (uint64_t)x->grid);
    HIPCHK(hipEventRecord(s.evm, x->stream));  // (re-recorded after the level kernel)
    HIPCHK(launch_expand(L, cur_ring(x, s), 0, s.n_cur, s.cur_base, next_ring(x, s), s.parents, next_base[0],
                         next_cap[0], s.table, x->tlog2, s.ctr, box, grid, x->stream, env_xflags(), nullptr, s.evm));
  } else {
    // Exchange rounds.  Each round every shard requeues its overflow list,
    // expands the rest of its frontier until an owner region of its outbox
    // fills (or, without the group guard, x->chunk states), and the records
    // travel (gather_counts .. k_build_winners).  Every rank learns from the
    // round's count gather what every shard has left, so all issue the same
    // collectives, and the rounds end together once nothing is left.
    for (auto& s : x->sh) {
      s.pos = 0;
      s.over_n = 0;
    }
    uint64_t last_left = ~0ull;
    for (uint64_t round = 0;; round++) {
      for (size_t k = 0; k < x->sh.size(); k++) {
        Shard& s = x->sh[k];
        const int nv = s.ov ^ 1;  // the overflow list this round appends to
        HIPCHK(hipMemsetAsync(s.out_count, 0, 8 * G, x->stream));
        HIPCHK(hipMemsetAsync(s.over_cnt + nv, 0, 8, x->stream));
        ShardBox box{G, s.id, (unsigned long long)x->box_cap, x->slog2, (unsigned long long*)s.out_count,
                     (unsigned long long*)s.send_fp, (unsigned long long*)s.send_ref,
                     (unsigned long long)x->stop_at, (unsigned long long*)s.over_fp[nv],
                     (unsigned long long*)s.over_ref[nv], (unsigned long long*)(s.over_cnt + nv),
                     (unsigned long long)x->over_cap};
        HIPCHK(launch_requeue(s.over_fp[s.ov], s.over_ref[s.ov], s.over_cnt + s.ov, s.over_n, box, s.ctr, x->stream));
        const uint64_t b = s.pos, e = x->chunk ? std::min<uint64_t>(s.n_cur, b + x->chunk) : s.n_cur;
        if (e > b) {
          uint64_t blocks = (e - b + 3) / 4;
          int grid = (int)std::min<uint64_t>(std::max<uint64_t>(blocks, 1), (uint64_t)x->grid);
          HIPCHK(launch_expand(L, cur_ring(x, s), b, e, s.cur_base, next_ring(x, s), s.parents, next_base[k],
                               next_cap[k], s.table, x->tlog2, s.ctr, box, grid, x->stream, env_xflags(), s.sent));
        }
        HIPCHK(launch_round_tail(s.ctr, s.out_count, G, e - b, s.n_cur - e, x->guarded && e > b, s.over_cnt + nv,
                                 x->stream));
        s.ov = nv;
      }
      if (round == 0 && fault_here(x, "exchange")) lflags |= FLAG_LOCAL_FAILURE;
      int rc = gather_counts(x);
      if (rc) return rc;
      const int RW = G + 2;
      uint64_t left = 0, sent_recs = 0;  // frontier states and overflow records left anywhere, records this round
      for (int r = 0; r < G; r++) {
        left += x->h_rows[(size_t)r * RW + G] + x->h_rows[(size_t)r * RW + G + 1];
        for (int p = 0; p < G; p++) sent_recs += x->h_rows[(size_t)r * RW + p];
      }
      for (auto& s : x->sh) {
        s.pos = s.n_cur - x->h_rows[(size_t)s.id * RW + G];
        s.over_n = x->h_rows[(size_t)s.id * RW + G + 1];
        x->overflowed += s.over_n;
        for (int p = 0; p < G; p++) x->records += s.h_out[p];
      }
      x->rounds++;
      if (left && !sent_recs && left >= last_left) {  // (cannot happen: a round with room takes a group)
        fprintf(stderr, "rtla: exchange round %llu made no progress\n", (unsigned long long)round);
        report_flags(FLAG_OUTBOX_FULL);
        x->finished = true;
        return RTLA_E_OVERFLOW;
      }
      last_left = left;
      rc = move_fps(x);
      if (rc) return rc;
      for (auto& s : x->sh) {
        uint64_t mx_in = 0;
        for (int p = 0; p < G; p++) mx_in = std::max(mx_in, s.h_in[p]);
        HIPCHK(launch_insert_remote(s.recv_fp, s.in_count, G, x->box_cap, s.table, x->tlog2, s.recv_ans, s.ctr, mx_in,
                                    x->stream));
      }
      rc = move_answers(x);
      if (rc) return rc;
      for (size_t k = 0; k < x->sh.size(); k++) {  // each sender builds its winners into its own next level
        Shard& s = x->sh[k];
        uint64_t mx_out = 0;
        for (int p = 0; p < G; p++) mx_out = std::max(mx_out, s.h_out[p]);
        HIPCHK(launch_build_winners(L, cur_ring(x, s), s.cur_base, s.id, s.send_ref, s.send_ans, s.out_count, G,
                                    x->box_cap, next_ring(x, s), s.parents, next_base[k], next_cap[k], s.ctr, mx_out,
                                    x->stream));
      }
      if (!left) break;
    }
  }
  for (auto& s : x->sh) HIPCHK(hipEventRecord(s.ev1, x->stream));
  // gather counters
  // new, generated, probes, frontier, next-level states per shard (global id), then one count per flag bit
  // (bits are summed, not max-reduced: every rank then reports the union of the flags)
  constexpr int NFLAG = 8;
  uint64_t sums[4 + SHARD_MAX + NFLAG] = {};
  uint64_t maxs[4] = {0, 0, 0, 0};  // flags, violation, device time (us), largest next frontier of a shard
  double emax = 0.0;  // probe-kernel (k_expand_*) time of this level, ms
  std::vector<DevCounters> hc(x->sh.size());
  for (size_t k = 0; k < x->sh.size(); k++)
    HIPCHK(hipMemcpyAsync(&hc[k], x->sh[k].ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  for (size_t k = 0; k < x->sh.size(); k++) {
    Shard& s = x->sh[k];
    float kms = 0.f, ems = 0.f;
    (void)hipEventElapsedTime(&kms, s.ev0, s.ev1);
    if (G == 1) (void)hipEventElapsedTime(&ems, s.ev0, s.evm);
    else ems = kms;  // multi-shard: rows are built inside the exchange rounds
    emax = std::max(emax, (double)ems);
    sums[0] += hc[k].next_count; sums[1] += hc[k].generated; sums[2] += hc[k].probes; sums[3] += s.n_cur;
    sums[4 + s.id] = hc[k].next_count;
    lflags |= hc[k].flags;
    maxs[1] = std::max<uint64_t>(maxs[1], hc[k].viol_mask ? 1 : 0);
    maxs[2] = std::max<uint64_t>(maxs[2], (uint64_t)(kms * 1000.0));
    maxs[3] = std::max<uint64_t>(maxs[3], hc[k].next_count);
    if (hc[k].viol_mask && !s.viol_mask) {
      s.viol_mask = hc[k].viol_mask; s.viol_in_model = hc[k].viol_in_model; s.viol_inst = hc[k].viol_inst;
      s.viol_parent = hc[k].viol_parent; s.viol_child = hc[k].viol_child;
    }
  }
  print_stamps(hc[0], x->level + 1);
  const int nsum = 4 + (G > 1 ? G : 0);
  for (int b = 0; b < NFLAG; b++) sums[nsum + b] = (uint64_t)(lflags >> b & 1);
  int rc = allreduce2_u64(x, sums, nsum + NFLAG, maxs, 4);
  if (rc) return rc;
  for (int b = 0; b < NFLAG; b++)
    if (sums[nsum + b]) maxs[0] |= 1ull << b;
  x->max_front = maxs[3];
  if (maxs[0]) {
    report_flags((int)maxs[0]);
    x->finished = true;
    if (st) {  // the level is incomplete: only which capacity ran out is reported
      memset(st, 0, sizeof *st);
      st->level = x->level + 1; st->status = flags_to_status((int)maxs[0]); st->flags = (int32_t)maxs[0];
      st->frontier = sums[3]; st->distinct_total = x->distinct; st->generated_total = x->generated;
      st->row_bytes = (uint64_t)L.W * 4; st->seconds = now_s() - t0;
    }
    return flags_to_status((int)maxs[0]);
  }
  uint64_t nnew = sums[0];
  x->generated += sums[1];
  x->distinct += nnew;
  x->level++;
  int status = RTLA_OK;
  if (maxs[1]) {
    x->finished = true;
    status = RTLA_VIOLATION;
  } else if (nnew == 0) {
    x->finished = true;
    status = RTLA_DONE;
  }
  std::vector<uint64_t> nnext(sums + 4, sums + 4 + G);
  if (G > 1 && status == RTLA_OK) {  // even out the shards' next levels (rows stay with their senders)
    if (int r = rebalance(x, nnext, next_base, next_cap)) return r;
    x->max_front = *std::max_element(nnext.begin(), nnext.end());
  }
  for (size_t k = 0; k < x->sh.size(); k++) {
    Shard& s = x->sh[k];
    s.cur_base = next_base[k];
    s.cur_start = next_ring(x, s).start;
    s.n_cur = G > 1 ? nnext[s.id] : hc[k].next_count;
  }
  if (st) {
    memset(st, 0, sizeof *st);
    st->level = x->level; st->status = status; st->frontier = sums[3]; st->new_states = nnew;
    st->generated = sums[1]; st->distinct_total = x->distinct; st->generated_total = x->generated;
    st->kernel_ms = maxs[2] / 1000.0; st->probes = sums[2]; st->row_bytes = (uint64_t)L.W * 4;
    st->expand_ms = x->world > 1 ? st->kernel_ms : emax;
    st->seconds = now_s() - t0;
  }
  return status;
}

static Shard* viol_shard(rtla_ctx* x) {  // violation found on a local shard
  for (auto& s : x->sh)
    if (s.viol_mask) return &s;
  return nullptr;
}

extern "C" int rtla_violation(rtla_ctx* x, int32_t* inv_mask, int32_t* in_model) {
  if (!x) return RTLA_E_ARG;
  Shard* s = viol_shard(x);
  if (inv_mask) *inv_mask = s ? s->viol_mask : 0;
  if (in_model) *in_model = s ? s->viol_in_model : 0;
  return s ? RTLA_VIOLATION : RTLA_OK;
}

extern "C" int rtla_frontier(rtla_ctx* x, uint32_t* rows, size_t cap, size_t* n) {
  if (!x || !n) return RTLA_E_ARG;
  if (!x->inited) return RTLA_E_STATE;
  size_t tot = 0;
  for (auto& s : x->sh) tot += s.n_cur;
  *n = tot;
  if (!rows) return RTLA_OK;
  if (tot > cap) return RTLA_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  size_t off = 0;
  for (auto& s : x->sh) {
    if (s.n_cur)
      HIPCHK(ring_copy(cur_ring(x, s), x->L.W, 0, s.n_cur, rows + off * x->L.W, true));
    off += s.n_cur;
  }
  return RTLA_OK;
}

// Digest of the current frontier: rows stream to the host in chunks (the
// next chunk's copy overlaps the current chunk's hashing).
static int level_digest(rtla_ctx* x, int threads, uint64_t* out, bool orbit) {
  if (!x || !out) return RTLA_E_ARG;
  if (!x->inited) return RTLA_E_STATE;
  // A local failure (device, pinned buffers, a copy) skips the hashing but
  // still reaches the reduction below, so no other rank waits in it.
  int rc = hipSetDevice(x->device) == hipSuccess ? RTLA_OK : RTLA_E_HIP;
  const int W = x->L.W;
  const int nt = text_threads(threads);
  const uint64_t CH = std::max<uint64_t>(1, (256ull << 20) / (4ull * W));  // ~256 MB of rows per chunk
  uint32_t* hbuf[2] = {nullptr, nullptr};
  for (auto& b : hbuf)
    if (!rc && hipHostMalloc((void**)&b, CH * W * 4, hipHostMallocDefault) != hipSuccess) {
      b = nullptr;
      rc = RTLA_E_HIP;
    }
  uint64_t sum = 0;
  for (auto& s : x->sh) {
    if (rc) break;
    const Ring r = cur_ring(x, s);
    // chunk j covers states [j * CH, ...); copies go in pieces that do not wrap the ring
    auto issue = [&](uint64_t g0, uint32_t* dst) -> hipError_t {
      uint64_t n = std::min<uint64_t>(CH, s.n_cur - g0), g = g0;
      while (n) {
        const uint64_t p = ring_idx(r, g), m = std::min<uint64_t>(n, r.cap - p);
        hipError_t e = hipMemcpyAsync(dst, r.base + p * (uint64_t)W, m * W * 4, hipMemcpyDeviceToHost, x->stream);
        if (e != hipSuccess) return e;
        dst += m * (uint64_t)W;
        g += m;
        n -= m;
      }
      return hipSuccess;
    };
    if (!s.n_cur) continue;
    if (issue(0, hbuf[0]) != hipSuccess) { rc = RTLA_E_HIP; break; }
    for (uint64_t g = 0, j = 0; g < s.n_cur; g += CH, j++) {
      if (hipStreamSynchronize(x->stream) != hipSuccess) { rc = RTLA_E_HIP; break; }
      if (g + CH < s.n_cur && issue(g + CH, hbuf[(j + 1) & 1]) != hipSuccess) { rc = RTLA_E_HIP; break; }
      sum += rows_digest(x->L, hbuf[j & 1], std::min<uint64_t>(CH, s.n_cur - g), nt, orbit);
    }
    if (rc) break;
  }
  (void)hipStreamSynchronize(x->stream);
  for (auto& b : hbuf)
    if (b) (void)hipHostFree(b);
  // every rank joins the reduction, also after a local failure (the flag travels with it)
  uint64_t v[2] = {sum, rc ? 1ull : 0ull};
  if (int e = allreduce_u64(x, v, 2, 0)) return e;
  if (rc) return rc;
  if (v[1]) return RTLA_E_HIP;
  *out = v[0];
  return RTLA_OK;
}

extern "C" int rtla_level_text_hash(rtla_ctx* x, int threads, uint64_t* out) {
  return level_digest(x, threads, out, false);
}
extern "C" int rtla_level_orbit_hash(rtla_ctx* x, int threads, uint64_t* out) {
  return level_digest(x, threads, out, true);
}

// Collective when world > 1: a local failure (device, read-back) travels in
// the reduction (its last word), so every rank fails together.
extern "C" int rtla_coverage(rtla_ctx* x, uint64_t* gen, uint64_t* distinct, int n) {
  if (!x) return RTLA_E_ARG;
  std::vector<uint64_t> acc(2 * COVER_CODES + 1, 0);
  bool bad = hipSetDevice(x->device) != hipSuccess || fault_here(x, "coverage");
  for (auto& s : x->sh) {
    DevCounters h;
    if (bad || hipMemcpy(&h, s.ctr, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) {
      bad = true;
      break;
    }
    for (int k = 0; k < 2 * COVER_CODES; k++) acc[k] += h.cover[k];
  }
  acc[2 * COVER_CODES] = bad ? 1 : 0;
  int rc = allreduce_u64(x, acc.data(), 2 * COVER_CODES + 1, 0);
  if (rc) return rc;
  if (acc[2 * COVER_CODES]) return bad ? RTLA_E_HIP : RTLA_E_COMM;
  for (int k = 0; k < n && k < COVER_CODES; k++) {
    if (gen) gen[k] = acc[k];
    if (distinct) distinct[k] = acc[COVER_CODES + k];
  }
  return COVER_CODES;
}

// Counterexample: find the violating state (or its parent + action when the
// violation was seen before the state had a home), walk the parent records
// back to Init -- across shards: a record is shard << 56 | index << 16 |
// instance -- then replay the action instances forward from the Init row with
// the kernel that built them.  Collective when world > 1 (every rank calls it;
// each step's record is broadcast by the rank that holds it).
extern "C" int rtla_trace(rtla_ctx* x, uint32_t* rows, int32_t* labels, size_t cap, size_t* n_rows) {
  if (!x || !n_rows) return RTLA_E_ARG;
  // world > 1: every rank reaches every reduction below; a local failure
  // travels in them (a failure count), so all ranks stop at the same step
  bool bad = hipSetDevice(x->device) != hipSuccess || fault_here(x, "trace");
  if (bad && x->world == 1) return RTLA_E_HIP;
  const Layout& L = x->L;
  // start: (holder shard, shard-local index, pending instance or -1)
  uint64_t start[4] = {0, 0, 0, 0};  // has, shard, g, inst + 1
  Shard* vs = nullptr;
  for (auto& s : x->sh)
    if (s.viol_mask) { vs = &s; break; }
  if (vs) {
    start[0] = 1;
    start[1] = (uint64_t)vs->id;
    if (vs->viol_inst < 0) { start[2] = 0; start[3] = 0; }
    else if (vs->viol_in_model && vs->viol_child != ~0ull) { start[2] = vs->viol_child; start[3] = 0; }
    else { start[2] = vs->viol_parent; start[3] = (uint64_t)vs->viol_inst + 1; }
  }
  if (x->world > 1) {
    // the lowest shard holding a violation publishes its start record
    uint64_t v[2] = {(uint64_t)x->nshard - (start[0] ? start[1] : (uint64_t)x->nshard), bad ? 1ull : 0ull};
    int rc = allreduce_u64(x, v, 2, 1);  // max of (G - holder) == min holder; any failure
    if (rc) return rc;
    if (v[1]) return bad ? RTLA_E_HIP : RTLA_E_COMM;
    if (v[0] == 0) return RTLA_E_STATE;
    const int root = (int)((uint64_t)x->nshard - v[0]);
    uint64_t w[5] = {0, 0, 0, 0, 0};  // root's start record, then the failure count
    if (x->rank == root) memcpy(w, start, 32);
    rc = allreduce_u64(x, w, 5, 0);
    if (rc) return rc;
    memcpy(start, w, 32);
  } else if (!start[0]) {
    return RTLA_E_STATE;
  }
  std::vector<int32_t> insts;
  if (start[3]) insts.push_back((int32_t)(start[3] - 1));
  uint64_t shard = start[1], g = start[2];
  for (int guard = 0; guard < (1 << 20); guard++) {
    uint64_t p = 0;
    if (x->world == 1 && !x->rccl_local) {
      HIPCHK(hipMemcpy(&p, x->sh[shard].parents + g, 8, hipMemcpyDeviceToHost));
    } else if (x->world == 1) {  // the record travels through the one-rank communicator too
      HIPCHK(hipMemcpyAsync(x->red, x->sh[shard].parents + g, 8, hipMemcpyDeviceToDevice, x->stream));
      if (int rc2 = comm_bcast(x, x->red, 1, 0)) return rc2;
      HIPCHK(hipMemcpyAsync(&p, x->red, 8, hipMemcpyDeviceToHost, x->stream));
      HIPCHK(hipStreamSynchronize(x->stream));
    } else {
      // the holder contributes the record, every rank its failure flag
      uint64_t w[2] = {0, 0};
      if ((int)shard == x->rank && !bad && hipMemcpy(&w[0], x->sh[0].parents + g, 8, hipMemcpyDeviceToHost) != hipSuccess)
        bad = true;
      w[1] = bad ? 1 : 0;
      if ((int)shard == x->rank && bad) w[0] = 0;
      if (int rc2 = allreduce_u64(x, w, 2, 0)) return rc2;
      if (w[1]) return bad ? RTLA_E_HIP : RTLA_E_COMM;
      p = w[0];
    }
    if (p == ~0ull) break;  // Init
    insts.push_back((int32_t)(p & 0xffff));
    shard = p >> 56;
    g = (p >> 16) & ((1ull << 40) - 1);
  }
  std::reverse(insts.begin(), insts.end());
  size_t n = insts.size() + 1;
  *n_rows = n;
  if (!rows && !labels) return RTLA_OK;
  if (n > cap) return RTLA_E_ARG;
  std::vector<uint32_t> row = x->init_row;
  uint32_t* d_row = nullptr;
  HIPCHK(hipMalloc(&d_row, 64 * L.W * 4));  // a whole 64-row group (the level kernel's tile)
  if (rows) memcpy(rows, row.data(), L.W * 4);
  if (labels) labels[0] = -1;
  int rc = RTLA_OK;
  for (size_t k = 0; k < insts.size() && rc == RTLA_OK; k++) {
    if (hipMemcpy(d_row, row.data(), L.W * 4, hipMemcpyHostToDevice) != hipSuccess) { rc = RTLA_E_HIP; break; }
    std::vector<uint32_t> out;
    std::vector<uint64_t> info;
    int r = expand_batch_dev(L, d_row, 1, out, info, x->stream);
    if (r < 0) { rc = r; break; }
    size_t hit = info.size();
    for (size_t q = 0; q < info.size(); q++)
      if ((int32_t)(info[q] & 0xffff) == insts[k]) hit = q;
    if (hit == info.size()) { rc = RTLA_E_STATE; break; }
    memcpy(row.data(), &out[hit * L.W], L.W * 4);
    if (rows) memcpy(rows + (k + 1) * L.W, row.data(), L.W * 4);
    if (labels) labels[k + 1] = (int32_t)(info[hit] & 0x7fffffffu);
  }
  (void)hipFree(d_row);
  return rc;
}

// Synthetic microbench step (BASELINE configs[4]): generate input states
// [first, first + n) into the row arena on the device (k_random_rows), then
// one launch of the level kernel over them in dedup-only mode: Next,
// fingerprint, probe/insert into this context's fingerprint set, no rows kept.
// The set accumulates across calls (rtla_reset clears it).
extern "C" int rtla_synthetic_generate(rtla_ctx* x, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool,
                                       uint64_t at) {
  if (!x) return RTLA_E_ARG;
  if (x->sh.size() != 1 || x->nshard != 1 || x->inited) return RTLA_E_STATE;
  if (at > x->front_cap || n > x->front_cap - at) return RTLA_E_OVERFLOW;
  HIPCHK(hipSetDevice(x->device));
  Shard& s = x->sh[0];
  HIPCHK(launch_random_rows(x->L, seed, first, n, pool, s.arena + at * (uint64_t)x->L.W, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  return RTLA_OK;
}

// One dedup-only level-kernel launch over arena rows [begin, end).
extern "C" int rtla_synthetic_dedup(rtla_ctx* x, uint64_t begin, uint64_t end, rtla_level_stats* st) {
  if (!x || !st || begin > end || begin % 64) return RTLA_E_ARG;  // level-kernel groups start at multiples of 64
  if (x->sh.size() != 1 || x->nshard != 1 || x->inited) return RTLA_E_STATE;
  if (end > x->front_cap) return RTLA_E_OVERFLOW;
  const double t0 = now_s();
  HIPCHK(hipSetDevice(x->device));
  Shard& s = x->sh[0];
  HIPCHK(hipMemsetAsync(s.ctr, 0, offsetof(DevCounters, cover), x->stream));
  s.h_caps[0] = end; s.h_caps[1] = 0; s.h_caps[2] = s.parents_cap;
  HIPCHK(hipMemcpyAsync(&s.ctr->cap_cur, s.h_caps, sizeof s.h_caps, hipMemcpyHostToDevice, x->stream));
  const Ring ring{s.arena, 0, x->front_cap};
  ShardBox box{1, 0, 0, 0, nullptr, nullptr, nullptr};
  HIPCHK(hipEventRecord(s.ev0, x->stream));
  HIPCHK(launch_expand(x->L, ring, begin, end, 0, ring, s.parents, 0, 0, s.table, x->tlog2, s.ctr, box, x->grid,
                       x->stream, env_xflags() | XF_DEDUP_ONLY));
  HIPCHK(hipEventRecord(s.ev1, x->stream));
  DevCounters h;
  HIPCHK(hipMemcpyAsync(&h, s.ctr, sizeof h, hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, s.ev0, s.ev1));
  print_stamps(h, 0);
  memset(st, 0, sizeof *st);
  st->frontier = end - begin; st->new_states = h.next_count; st->generated = h.generated; st->probes = h.probes;
  st->kernel_ms = ms; st->expand_ms = ms; st->row_bytes = (uint64_t)x->L.W * 4; st->flags = h.flags;
  st->seconds = now_s() - t0;
  if (h.flags) {
    report_flags(h.flags);
    return flags_to_status(h.flags);
  }
  return RTLA_OK;
}

extern "C" int rtla_synthetic_step(rtla_ctx* x, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool,
                                   rtla_level_stats* st) {
  if (!st) return RTLA_E_ARG;
  const int rc = rtla_synthetic_generate(x, seed, first, n, pool, 0);
  return rc < 0 ? rc : rtla_synthetic_dedup(x, 0, n, st);
}

// Diagnostic: re-expand the current frontier `reps` times with the given
// k_expand_lane switches (XF_*) and report the mean device time per launch.
// Successors are inserted into the fingerprint set (so later reps find them
// seen) and written to the idle frontier buffer: call it only at the end of
// a search, never between rtla_step calls whose results matter.
extern "C" int rtla_time_expand(rtla_ctx* x, int xflags, int reps, double* ms) {
  if (!x || reps < 1 || !ms) return RTLA_E_ARG;
  if (x->sh.size() != 1 || x->nshard != 1) return RTLA_E_STATE;
  HIPCHK(hipSetDevice(x->device));
  Shard& s = x->sh[0];
  const uint64_t next_base = s.cur_base + s.n_cur;
  if (next_base >= s.parents_cap) return RTLA_E_OVERFLOW;
  const uint64_t next_cap = std::min<uint64_t>(next_room(x, s), s.parents_cap - next_base);
  ShardBox box{1, 0, 0, 0, nullptr, nullptr, nullptr};
  float total = 0.f;
  for (int r = 0; r < reps; r++) {
    HIPCHK(hipMemsetAsync(s.ctr, 0, offsetof(DevCounters, cover), x->stream));
    HIPCHK(hipEventRecord(s.ev0, x->stream));
    HIPCHK(launch_expand(x->L, cur_ring(x, s), 0, s.n_cur, s.cur_base, next_ring(x, s), s.parents, next_base,
                         next_cap, s.table, x->tlog2, s.ctr, box, x->grid, x->stream, xflags));
    HIPCHK(hipEventRecord(s.ev1, x->stream));
    HIPCHK(hipEventSynchronize(s.ev1));
    float m = 0.f;
    HIPCHK(hipEventElapsedTime(&m, s.ev0, s.ev1));
    total += m;
  }
  *ms = total / reps;
  return RTLA_OK;
}

// Calibration of the fingerprint-set probe: n random keys inserted (all new,
// CAS), then the same n keys probed again (all present) with a CAS and with
// the load-first protocol the BFS kernel uses.  Device seconds of each pass.
extern "C" int rtla_probe_bench2(int log2, uint64_t n, double* s_insert, double* s_seen_cas, double* s_seen_load,
                                 uint64_t* inserted) {
  uint64_t* table = nullptr;
  DevCounters* ctr = nullptr;
  HIPCHK(hipMalloc(&table, 8ull << log2));
  HIPCHK(hipMalloc(&ctr, sizeof(DevCounters)));
  HIPCHK(hipMemset(table, 0, 8ull << log2));
  HIPCHK(hipMemset(ctr, 0, sizeof(DevCounters)));
  hipEvent_t e[4];
  for (auto& v : e) HIPCHK(hipEventCreate(&v));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipEventRecord(e[0], nullptr));
  HIPCHK(launch_probe_bench(table, log2, n, 777, ctr, nullptr, 0));
  HIPCHK(hipEventRecord(e[1], nullptr));
  HIPCHK(launch_probe_bench(table, log2, n, 777, ctr, nullptr, 0));
  HIPCHK(hipEventRecord(e[2], nullptr));
  HIPCHK(launch_probe_bench(table, log2, n, 777, ctr, nullptr, 1));
  HIPCHK(hipEventRecord(e[3], nullptr));
  HIPCHK(hipEventSynchronize(e[3]));
  float ms[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) HIPCHK(hipEventElapsedTime(&ms[k], e[k], e[k + 1]));
  DevCounters h;
  HIPCHK(hipMemcpy(&h, ctr, sizeof h, hipMemcpyDeviceToHost));
  if (s_insert) *s_insert = ms[0] / 1e3;
  if (s_seen_cas) *s_seen_cas = ms[1] / 1e3;
  if (s_seen_load) *s_seen_load = ms[2] / 1e3;
  if (inserted) *inserted = h.next_count;  // the two re-probe passes insert nothing
  for (auto& v : e) (void)hipEventDestroy(v);
  (void)hipFree(table);
  (void)hipFree(ctr);
  return RTLA_OK;
}

extern "C" int rtla_probe_bench3(int log2, uint64_t n_present, uint64_t n, double new_frac, double* seconds,
                                 uint64_t* inserted) {
  if (log2 < 16 || log2 > 36 || !n || n_present >= (1ull << log2)) return RTLA_E_ARG;
  uint64_t* table = nullptr;
  DevCounters* ctr = nullptr;
  HIPCHK(hipMalloc(&table, 8ull << log2));
  int rc = RTLA_OK;
  if (hipMalloc(&ctr, sizeof(DevCounters)) != hipSuccess) rc = RTLA_E_HIP;
  hipEvent_t e[2] = {nullptr, nullptr};
  float ms = 0.f;
  DevCounters h;
  memset(&h, 0, sizeof h);
  auto step = [&](hipError_t v) {
    if (!rc && v != hipSuccess) rc = RTLA_E_HIP;
  };
  step(hipMemset(table, 0, 8ull << log2));
  if (!rc) step(hipMemset(ctr, 0, sizeof(DevCounters)));
  for (auto& v : e)
    if (!rc) step(hipEventCreate(&v));
  if (!rc) step(launch_probe_bench(table, log2, n_present, 777, ctr, nullptr, 0));  // the present keys (untimed)
  if (!rc) step(hipMemset(ctr, 0, sizeof(DevCounters)));
  if (!rc) step(hipDeviceSynchronize());
  if (!rc) step(hipEventRecord(e[0], nullptr));
  if (!rc) step(launch_probe_mixed(table, log2, n, n_present, new_frac, 777, ctr, nullptr));
  if (!rc) step(hipEventRecord(e[1], nullptr));
  if (!rc) step(hipEventSynchronize(e[1]));
  if (!rc) step(hipEventElapsedTime(&ms, e[0], e[1]));
  if (!rc) step(hipMemcpy(&h, ctr, sizeof h, hipMemcpyDeviceToHost));
  if (!rc && (h.flags & FLAG_FPSET_FULL)) rc = RTLA_E_OVERFLOW;
  if (seconds) *seconds = ms / 1e3;
  if (inserted) *inserted = h.next_count;
  for (auto& v : e)
    if (v) (void)hipEventDestroy(v);
  (void)hipFree(table);
  if (ctr) (void)hipFree(ctr);
  return rc;
}

extern "C" int rtla_probe_bench(int log2, uint64_t n, double* seconds, uint64_t* inserted) {
  uint64_t* table = nullptr;
  DevCounters* ctr = nullptr;
  HIPCHK(hipMalloc(&table, 8ull << log2));
  HIPCHK(hipMalloc(&ctr, sizeof(DevCounters)));
  HIPCHK(hipMemset(table, 0, 8ull << log2));
  HIPCHK(hipMemset(ctr, 0, sizeof(DevCounters)));
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  HIPCHK(launch_probe_bench(table, log2, n / 8, 12345, ctr, nullptr));  // warm
  HIPCHK(hipMemset(table, 0, 8ull << log2));
  HIPCHK(hipMemset(ctr, 0, sizeof(DevCounters)));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipEventRecord(a, nullptr));
  HIPCHK(launch_probe_bench(table, log2, n, 777, ctr, nullptr));
  HIPCHK(hipEventRecord(b, nullptr));
  HIPCHK(hipEventSynchronize(b));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  DevCounters h;
  HIPCHK(hipMemcpy(&h, ctr, sizeof h, hipMemcpyDeviceToHost));
  if (seconds) *seconds = ms / 1e3;
  if (inserted) *inserted = h.next_count;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(table);
  (void)hipFree(ctr);
  return RTLA_OK;
}
