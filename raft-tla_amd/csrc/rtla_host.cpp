// rtla_host.cpp -- the C-ABI driver (include/rtla.h) around the HIP kernels.
//
// One context = one rank = one GPU.  Device memory per context:
//   fingerprint set   2^fpset_log2 x 8 B   (open addressing, CAS insert)
//   parents           one u64 per distinct state: parent global index << 16 | instance
//   frontier A / B    frontier_cap rows each (double buffer, swapped per level)
//   counters          DevCounters
// The level loop is host-driven: one k_expand launch per BFS level, then an
// 8-byte-scale counter read-back decides termination (TLC's "0 states left on
// queue").
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/rtla.h"
#include "rtla_device.h"
#include "rtla_launch.h"
#include "rtla_model.h"
#include "rtla_text.h"

using namespace rtla;

struct rtla_ctx {
  rtla_cfg cfg;
  Layout L;
  int rank = 0, world = 1, device = 0;
  hipStream_t stream = nullptr;
  uint64_t* table = nullptr;
  int tlog2 = 0;
  uint64_t* parents = nullptr;
  uint64_t parents_cap = 0;
  uint32_t* front[2] = {nullptr, nullptr};
  uint64_t front_cap = 0;
  int cur = 0;
  uint64_t n_cur = 0, cur_base = 0;
  DevCounters* ctr = nullptr;
  int* dflags = nullptr;
  int level = 0;
  bool inited = false, finished = false;
  uint64_t distinct = 0, generated = 0;
  int viol_mask = 0, viol_in_model = 0, viol_inst = -1;
  uint64_t viol_parent = 0, viol_child = ~0ull;
  int grid = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<uint32_t> init_row;
};

#define HIPCHK(x)                                                     \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "rtla: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return RTLA_E_HIP;                                              \
    }                                                                 \
  } while (0)

static int layout_from_cfg(const rtla_cfg* c, Layout* L) {
  if (!c) return RTLA_E_ARG;
  if (c->symmetry) return RTLA_E_CONFIG;
  int K = c->bag_cap ? c->bag_cap : (c->max_msgs > 0 ? c->max_msgs + 1 : 32);
  int E = c->elec_cap ? c->elec_cap : (c->max_term - 1) * c->n_server;
  if (E < 1) E = 1;
  if (make_layout(L, c->n_server, c->n_value, c->max_term, c->max_log, c->max_copies, c->max_msgs,
                  K, E, c->inv_mask) != 0)
    return RTLA_E_CONFIG;
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
    case RTLA_E_OVERFLOW: return "capacity overflow (bag/elections/frontier/fingerprint set)";
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
  return check_invariants(L, row, (const Delta*)nullptr);
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

static int flags_to_status(int flags) {
  if (flags & FLAG_SPEC_ERROR) return RTLA_E_SPEC;
  if (flags) return RTLA_E_OVERFLOW;
  return RTLA_OK;
}

static void report_flags(int flags) {
  if (flags & FLAG_SPEC_ERROR) fprintf(stderr, "rtla: TLC evaluation error in Next (sequence index outside DOMAIN)\n");
  if (flags & FLAG_ROW_OVERFLOW) fprintf(stderr, "rtla: row capacity exceeded (raise bag_cap / elec_cap)\n");
  if (flags & FLAG_FRONTIER_FULL) fprintf(stderr, "rtla: next-frontier buffer full (raise frontier_cap / mem_budget)\n");
  if (flags & FLAG_FPSET_FULL) fprintf(stderr, "rtla: fingerprint set too full (raise fpset_log2)\n");
}

// Run k_expand_batch on device rows; results copied to host vectors.
static int expand_batch_dev(const Layout& L, const uint32_t* d_rows, size_t n, std::vector<uint32_t>& out,
                            std::vector<uint64_t>& info, hipStream_t st) {
  size_t cap = n * (size_t)L.fam[F_COUNT];
  uint32_t* d_out = nullptr;
  uint64_t* d_info = nullptr;
  DevCounters* d_ctr = nullptr;
  HIPCHK(hipMalloc(&d_out, std::max<size_t>(cap, 1) * L.W * 4));
  HIPCHK(hipMalloc(&d_info, std::max<size_t>(cap, 1) * 8));
  HIPCHK(hipMalloc(&d_ctr, sizeof(DevCounters)));
  HIPCHK(hipMemsetAsync(d_ctr, 0, sizeof(DevCounters), st));
  HIPCHK(launch_expand_batch(L, d_rows, n, d_out, d_info, cap, d_ctr, st));
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
  hipFree(d_out); hipFree(d_info); hipFree(d_ctr);
  // canonical order: (input, instance)
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

extern "C" int rtla_expand_batch(const rtla_cfg* c, const uint32_t* rows, size_t n, uint32_t* succ,
                                 uint64_t* info, size_t cap, size_t* n_out) {
  Layout L;
  int r = layout_from_cfg(c, &L);
  if (r) return r;
  if (!rows || !n_out) return RTLA_E_ARG;
  uint32_t* d_rows = nullptr;
  HIPCHK(hipMalloc(&d_rows, std::max<size_t>(n, 1) * L.W * 4));
  HIPCHK(hipMemcpy(d_rows, rows, n * L.W * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> out;
  std::vector<uint64_t> inf;
  r = expand_batch_dev(L, d_rows, n, out, inf, nullptr);
  hipFree(d_rows);
  if (r < 0) return r;
  *n_out = inf.size();
  if (inf.size() > cap) return RTLA_E_ARG;
  if (succ) memcpy(succ, out.data(), out.size() * 4);
  if (info) memcpy(info, inf.data(), inf.size() * 8);
  return RTLA_OK;
}

extern "C" int rtla_comm_id(void* out128) {
  (void)out128;
  return RTLA_E_COMM;  // multi-rank contexts: see rtla_dist.cpp (not in this build)
}

extern "C" int rtla_open(const rtla_cfg* cfg, int rank, int world, const void* comm_id, rtla_ctx** out) {
  (void)comm_id;
  if (!cfg || !out) return RTLA_E_ARG;
  *out = nullptr;
  if (world != 1) return RTLA_E_CONFIG;
  rtla_ctx* x = new rtla_ctx();
  x->cfg = *cfg;
  int r = layout_from_cfg(cfg, &x->L);
  if (r) { delete x; return r; }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) { delete x; return RTLA_E_HIP; }
  x->rank = rank; x->world = world; x->device = rank % ndev;
  if (hipSetDevice(x->device) != hipSuccess) { delete x; return RTLA_E_HIP; }
  if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) { delete x; return RTLA_E_HIP; }
  size_t free_b = 0, total_b = 0;
  hipMemGetInfo(&free_b, &total_b);
  uint64_t budget = cfg->mem_budget ? cfg->mem_budget : (uint64_t)(free_b * 0.85);
  const Layout& L = x->L;
  // fingerprint set: <= 40% of the budget, power of two
  int tl = cfg->fpset_log2;
  if (!tl) {
    tl = 20;
    while (tl < 34 && (8ull << (tl + 1)) <= budget * 2 / 5) tl++;
  }
  if (tl < 10 || tl > 40) { rtla_close(x); return RTLA_E_CONFIG; }
  x->tlog2 = tl;
  uint64_t tbytes = 8ull << tl;
  x->parents_cap = (1ull << tl) - (1ull << tl) / 4;  // load factor <= 0.75
  uint64_t pbytes = x->parents_cap * 8;
  uint64_t rowb = (uint64_t)L.W * 4;
  uint64_t fcap = cfg->frontier_cap;
  if (!fcap) {
    uint64_t rest = budget > tbytes + pbytes ? budget - tbytes - pbytes : 0;
    fcap = rest / (2 * rowb);
  }
  if (fcap < 1024) fcap = 1024;
  x->front_cap = fcap;
  if (hipMalloc(&x->table, tbytes) != hipSuccess || hipMalloc(&x->parents, pbytes) != hipSuccess ||
      hipMalloc(&x->front[0], fcap * rowb) != hipSuccess || hipMalloc(&x->front[1], fcap * rowb) != hipSuccess ||
      hipMalloc(&x->ctr, sizeof(DevCounters)) != hipSuccess || hipMalloc(&x->dflags, sizeof(int) * 64) != hipSuccess) {
    fprintf(stderr, "rtla: device allocation failed (table %llu B, parents %llu B, frontier 2x%llu B)\n",
            (unsigned long long)tbytes, (unsigned long long)pbytes, (unsigned long long)(fcap * rowb));
    rtla_close(x);
    return RTLA_E_HIP;
  }
  hipMemsetAsync(x->table, 0, tbytes, x->stream);
  hipMemsetAsync(x->ctr, 0, sizeof(DevCounters), x->stream);
  if (hipStreamSynchronize(x->stream) != hipSuccess) { rtla_close(x); return RTLA_E_HIP; }
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, x->device);
  x->grid = prop.multiProcessorCount * expand_blocks_per_cu(L) * 2;
  hipEventCreate(&x->ev0);
  hipEventCreate(&x->ev1);
  *out = x;
  return RTLA_OK;
}

extern "C" void rtla_close(rtla_ctx* x) {
  if (!x) return;
  hipSetDevice(x->device);
  if (x->table) hipFree(x->table);
  if (x->parents) hipFree(x->parents);
  if (x->front[0]) hipFree(x->front[0]);
  if (x->front[1]) hipFree(x->front[1]);
  if (x->ctr) hipFree(x->ctr);
  if (x->dflags) hipFree(x->dflags);
  if (x->ev0) hipEventDestroy(x->ev0);
  if (x->ev1) hipEventDestroy(x->ev1);
  if (x->stream) hipStreamDestroy(x->stream);
  delete x;
}

extern "C" int rtla_device_info(rtla_ctx* x, char* buf, size_t cap) {
  if (!x || !buf) return RTLA_E_ARG;
  hipDeviceProp_t p;
  HIPCHK(hipGetDeviceProperties(&p, x->device));
  snprintf(buf, cap, "{\"device\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"fpset_slots_log2\": %d, "
           "\"frontier_cap\": %llu, \"row_words\": %d, \"grid\": %d}",
           p.name, p.gcnArchName, p.multiProcessorCount, x->tlog2, (unsigned long long)x->front_cap,
           x->L.W, x->grid);
  return RTLA_OK;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

extern "C" int rtla_init(rtla_ctx* x, rtla_level_stats* st) {
  if (!x) return RTLA_E_ARG;
  if (x->inited) return RTLA_E_STATE;
  double t0 = now_s();
  HIPCHK(hipSetDevice(x->device));
  const Layout& L = x->L;
  x->init_row.assign(L.W, 0);
  row_init(L, x->init_row.data());
  HIPCHK(hipMemcpyAsync(x->front[0], x->init_row.data(), L.W * 4, hipMemcpyHostToDevice, x->stream));
  HIPCHK(launch_insert_rows(L, x->front[0], 1, x->table, x->tlog2, x->dflags, x->ctr, x->stream));
  uint64_t root = ~0ull;  // Init has no parent
  HIPCHK(hipMemcpyAsync(x->parents, &root, 8, hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  x->cur = 0; x->n_cur = 1; x->cur_base = 0;
  x->level = 1; x->distinct = 1; x->generated = 1; x->inited = true;
  int bad = check_invariants(L, x->init_row.data(), (const Delta*)nullptr);
  int status = RTLA_OK;
  if (bad) {
    x->viol_mask = bad; x->viol_in_model = 1; x->viol_child = 0; x->viol_inst = -1;
    x->finished = true;
    status = RTLA_VIOLATION;
  }
  if (st) {
    memset(st, 0, sizeof *st);
    st->level = 1; st->status = status; st->frontier = 0; st->new_states = 1; st->generated = 1;
    st->distinct_total = 1; st->generated_total = 1; st->seconds = now_s() - t0;
    st->row_bytes = (uint64_t)L.W * 4;
  }
  return status;
}

extern "C" int rtla_reset(rtla_ctx* x) {
  if (!x) return RTLA_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  HIPCHK(hipMemsetAsync(x->table, 0, 8ull << x->tlog2, x->stream));
  HIPCHK(hipMemsetAsync(x->ctr, 0, sizeof(DevCounters), x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  x->inited = false; x->finished = false; x->level = 0; x->distinct = 0; x->generated = 0;
  x->n_cur = 0; x->cur_base = 0; x->cur = 0;
  x->viol_mask = 0; x->viol_in_model = 0; x->viol_inst = -1; x->viol_parent = 0; x->viol_child = ~0ull;
  return RTLA_OK;
}

extern "C" int rtla_step(rtla_ctx* x, rtla_level_stats* st) {
  if (!x) return RTLA_E_ARG;
  if (!x->inited) return RTLA_E_STATE;
  if (x->finished) return x->viol_mask ? RTLA_VIOLATION : RTLA_DONE;
  double t0 = now_s();
  HIPCHK(hipSetDevice(x->device));
  const Layout& L = x->L;
  HIPCHK(hipMemsetAsync(x->ctr, 0, offsetof(DevCounters, cover), x->stream));
  uint64_t next_base = x->cur_base + x->n_cur;
  uint64_t next_cap = x->front_cap;
  if (next_base >= x->parents_cap) return RTLA_E_OVERFLOW;
  if (next_cap > x->parents_cap - next_base) next_cap = x->parents_cap - next_base;
  uint64_t blocks = (x->n_cur + 3) / 4;
  int grid = (int)std::min<uint64_t>(blocks, (uint64_t)x->grid);
  HIPCHK(hipEventRecord(x->ev0, x->stream));
  HIPCHK(launch_expand(L, x->front[x->cur], x->n_cur, x->cur_base, x->front[x->cur ^ 1], x->parents,
                       next_base, next_cap, x->table, x->tlog2, x->ctr, grid, x->stream));
  HIPCHK(hipEventRecord(x->ev1, x->stream));
  DevCounters h;
  HIPCHK(hipMemcpyAsync(&h, x->ctr, sizeof h, hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  if (h.flags) { report_flags(h.flags); x->finished = true; return flags_to_status(h.flags); }
  float kms = 0.f;
  hipEventElapsedTime(&kms, x->ev0, x->ev1);
  uint64_t nnew = h.next_count;
  x->generated += h.generated;
  x->distinct += nnew;
  x->level++;
  int status = RTLA_OK;
  if (h.viol_mask) {
    x->viol_mask = h.viol_mask; x->viol_in_model = h.viol_in_model; x->viol_inst = h.viol_inst;
    x->viol_parent = h.viol_parent; x->viol_child = h.viol_child;
    x->finished = true;
    status = RTLA_VIOLATION;
  } else if (nnew == 0) {
    x->finished = true;
    status = RTLA_DONE;
  }
  if (st) {
    memset(st, 0, sizeof *st);
    st->level = x->level; st->status = status; st->frontier = x->n_cur; st->new_states = nnew;
    st->generated = h.generated; st->distinct_total = x->distinct; st->generated_total = x->generated;
    st->kernel_ms = kms; st->probes = h.probes; st->row_bytes = (uint64_t)L.W * 4;
  }
  x->cur_base = next_base;
  x->n_cur = nnew;
  x->cur ^= 1;
  if (st) st->seconds = now_s() - t0;
  return status;
}

extern "C" int rtla_violation(rtla_ctx* x, int32_t* inv_mask, int32_t* in_model) {
  if (!x) return RTLA_E_ARG;
  if (inv_mask) *inv_mask = x->viol_mask;
  if (in_model) *in_model = x->viol_in_model;
  return x->viol_mask ? RTLA_VIOLATION : RTLA_OK;
}

extern "C" int rtla_frontier(rtla_ctx* x, uint32_t* rows, size_t cap, size_t* n) {
  if (!x || !n) return RTLA_E_ARG;
  if (!x->inited) return RTLA_E_STATE;
  *n = (size_t)x->n_cur;
  if (!rows) return RTLA_OK;
  if (x->n_cur > cap) return RTLA_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  HIPCHK(hipMemcpy(rows, x->front[x->cur], (size_t)x->n_cur * x->L.W * 4, hipMemcpyDeviceToHost));
  return RTLA_OK;
}

extern "C" int rtla_coverage(rtla_ctx* x, uint64_t* gen, uint64_t* distinct, int n) {
  if (!x) return RTLA_E_ARG;
  DevCounters h;
  HIPCHK(hipSetDevice(x->device));
  HIPCHK(hipMemcpy(&h, x->ctr, sizeof h, hipMemcpyDeviceToHost));
  for (int k = 0; k < n && k < COVER_CODES; k++) {
    if (gen) gen[k] = h.cover[k];
    if (distinct) distinct[k] = h.cover[COVER_CODES + k];
  }
  return COVER_CODES;
}

// Counterexample: walk parent pointers back to Init, then replay the action
// instances forward from the Init row with the same kernel that built them.
extern "C" int rtla_trace(rtla_ctx* x, uint32_t* rows, int32_t* labels, size_t cap, size_t* n_rows) {
  if (!x || !n_rows) return RTLA_E_ARG;
  if (!x->viol_mask) return RTLA_E_STATE;
  HIPCHK(hipSetDevice(x->device));
  const Layout& L = x->L;
  std::vector<int32_t> insts;  // forward order after reversal
  uint64_t g;
  if (x->viol_inst < 0) {
    g = 0;  // Init itself
  } else if (x->viol_in_model && x->viol_child != ~0ull) {
    g = x->viol_child;
  } else {
    insts.push_back(x->viol_inst);
    g = x->viol_parent;
  }
  while (g != 0) {
    uint64_t p;
    HIPCHK(hipMemcpy(&p, x->parents + g, 8, hipMemcpyDeviceToHost));
    insts.push_back((int32_t)(p & 0xffff));
    g = p >> 16;
  }
  std::reverse(insts.begin(), insts.end());
  size_t n = insts.size() + 1;
  *n_rows = n;
  if (n > cap) return RTLA_E_ARG;
  std::vector<uint32_t> row = x->init_row;
  uint32_t* d_row = nullptr;
  HIPCHK(hipMalloc(&d_row, L.W * 4));
  if (rows) memcpy(rows, row.data(), L.W * 4);
  if (labels) labels[0] = -1;
  for (size_t k = 0; k < insts.size(); k++) {
    HIPCHK(hipMemcpy(d_row, row.data(), L.W * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> out;
    std::vector<uint64_t> info;
    int r = expand_batch_dev(L, d_row, 1, out, info, x->stream);
    if (r < 0) { hipFree(d_row); return r; }
    size_t hit = info.size();
    for (size_t q = 0; q < info.size(); q++)
      if ((int32_t)(info[q] & 0xffff) == insts[k]) hit = q;
    if (hit == info.size()) { hipFree(d_row); return RTLA_E_STATE; }
    memcpy(row.data(), &out[hit * L.W], L.W * 4);
    if (rows) memcpy(rows + (k + 1) * L.W, row.data(), L.W * 4);
    if (labels) labels[k + 1] = (int32_t)(info[hit] & 0xffffffffu & ~(1u << 31));
  }
  hipFree(d_row);
  return RTLA_OK;
}

extern "C" int rtla_probe_bench(int log2, uint64_t n, double* seconds, uint64_t* inserted) {
  uint64_t* table = nullptr;
  DevCounters* ctr = nullptr;
  HIPCHK(hipMalloc(&table, 8ull << log2));
  HIPCHK(hipMalloc(&ctr, sizeof(DevCounters)));
  HIPCHK(hipMemset(table, 0, 8ull << log2));
  HIPCHK(hipMemset(ctr, 0, sizeof(DevCounters)));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  HIPCHK(launch_probe_bench(table, log2, n / 8, 12345, ctr, nullptr));  // warm
  HIPCHK(hipMemset(table, 0, 8ull << log2));
  HIPCHK(hipMemset(ctr, 0, sizeof(DevCounters)));
  HIPCHK(hipDeviceSynchronize());
  hipEventRecord(a, nullptr);
  HIPCHK(launch_probe_bench(table, log2, n, 777, ctr, nullptr));
  hipEventRecord(b, nullptr);
  HIPCHK(hipEventSynchronize(b));
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  DevCounters h;
  HIPCHK(hipMemcpy(&h, ctr, sizeof h, hipMemcpyDeviceToHost));
  if (seconds) *seconds = ms / 1e3;
  if (inserted) *inserted = h.next_count;
  hipEventDestroy(a); hipEventDestroy(b);
  hipFree(table); hipFree(ctr);
  return RTLA_OK;
}
