/* raft_cpu.h -- C ABI of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 * See raft_cpu.c for what it restates and where it may be used. */
#ifndef RAFT_CPU_H
#define RAFT_CPU_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ORC_INV_NO_TWO_LEADERS 1
#define ORC_INV_ELECTION_SAFETY 2
#define ORC_INV_LOG_MATCHING 4

#define ORC_MAX_LEVELS 1024
#define ORC_MAX_ACTIONS 16

enum { ORC_OK = 0, ORC_VIOLATION = 1, ORC_E_CONFIG = -1, ORC_E_OVERFLOW = -2, ORC_E_SPEC = -3, ORC_E_BUDGET = -4 };

typedef struct {
    int n_server, n_value, max_term, max_log, max_copies, inv_mask;
    int verbose;
    int max_msgs;           /* 0 = unbounded; else BagCardinality(messages) <= max_msgs */
    uint64_t max_distinct;  /* 0 = unlimited; stop with ORC_E_BUDGET beyond */
    int symmetry;           /* SYMMETRY Permutations(Server): count server-permutation orbits */
    int max_levels;         /* 0 = unlimited; else stop after this many levels (Init = 1).  The last
                               level's new states are counted, hashed and deduplicated but not kept,
                               so a prefix reaches one level further in the same memory */
} orc_cfg;

typedef struct {
    int n_levels, depth, violated, trace_len;
    uint64_t distinct, generated;
    uint64_t level_new[ORC_MAX_LEVELS];
    uint64_t level_gen[ORC_MAX_LEVELS];
    uint64_t level_text_hash[ORC_MAX_LEVELS];  /* sum of FNV-1a(text) over new states; SYMMETRY:
                                                  of each new orbit's orbit text (raft_cpu.c) */
    uint64_t coverage[ORC_MAX_ACTIONS];
    uint64_t max_msgs, max_state_bytes;
    double seconds;
    char *trace_text;   /* malloc'd; free with orc_free */
} orc_result;

int orc_bfs(const orc_cfg *c, int nthreads, int keep_trace, int text_hash, orc_result *r);
void orc_free(void *p);
uint64_t orc_text_hash(const char *t);

void *orc_walk_new(const orc_cfg *c);
void orc_walk_free(void *h);
long orc_walk_successors(void *h, char *buf, size_t cap);
int orc_walk_goto(void *h, const char *text);
long orc_walk_text(void *h, char *buf, size_t cap);
int orc_walk_inv(void *h);
long orc_walk_orbits(void *h, char *buf, size_t cap);

void *orc_dedup_new(const orc_cfg *c);
void orc_dedup_free(void *h);
int orc_dedup_texts(void *h, const char *texts, size_t n, int threads, uint64_t *out, double *seconds);

#ifdef __cplusplus
}
#endif
#endif
