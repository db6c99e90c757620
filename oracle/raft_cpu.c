/*
 * raft_cpu.c -- CPU restatement of raft.tla + TLC-style BFS.
 *
 * TEST INFRASTRUCTURE ONLY: this is the parity oracle and the CPU baseline
 * ("port") of the MI355X model checker.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It shares NO code with the
 * product (raft-tla_amd/csrc): its representation is an unpacked struct with a
 * sorted, canonical message bag, sorted elections and a sorted allLogs set, and
 * its seen-set is keyed by a 128-bit hash of the canonical serialisation.
 *
 * Every action below cites the raft.tla line it restates
 * (/root/reference/raft.tla, sha256 683a120a...6b81).  The state constraint and
 * invariants are the build's own definitions (specs/MC.tla), because the
 * reference's raft.cfg:3 names an undefined NoTwoLeaders and has no CONSTRAINT.
 *
 * Parity status: TLC cannot run here (no JVM) and the reference ships no
 * fixtures: this oracle is pinned by hand-derived KATs and by
 * agreement with the value-semantics oracle oracle/raft_values.py on small
 * configs ("parity unpinned" against TLC itself).
 *
 * Build: see oracle/Makefile (shared library + CLI).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "raft_cpu.h"

#define NMAX 5
#define LCAP 7      /* log length capacity (max_log + 1, out-of-model)   */
#define KMAX 255    /* distinct messages in one state                    */
#define EMAX 64     /* election records                                  */
#define AMAX 4096   /* logs in allLogs                                   */

enum { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum { RVREQ = 0, RVRESP = 1, AEREQ = 2, AERESP = 3 };
#define NIL 0xFF

/* A log is a u64: bits 0-3 length, entry k (1-based) in bits 4+8(k-1) as
 * term<<4 | value.  Equal logs <=> equal codes. */
typedef uint64_t Log;
static inline int log_len(Log l) { return (int)(l & 15); }
static inline int log_term(Log l, int k) { return (int)((l >> (4 + 8 * (k - 1) + 4)) & 15); }
static inline int log_val(Log l, int k) { return (int)((l >> (4 + 8 * (k - 1))) & 15); }
static inline Log log_append(Log l, int t, int v) {
    int n = log_len(l);
    return ((l & ~(Log)15) | (Log)(n + 1)) | ((Log)((t << 4) | v) << (4 + 8 * n));
}
static inline Log log_prefix(Log l, int n) {   /* SubSeq(l, 1, n) */
    Log body = (n == 0) ? 0 : ((l >> 4) & (((Log)1 << (8 * n)) - 1)) << 4;
    return body | (Log)n;
}
static inline int last_term(Log l) { int n = log_len(l); return n ? log_term(l, n) : 0; }

typedef struct {
    uint8_t type, term, src, dst;
    uint8_t a, b, c, d;     /* RVReq: a=lastLogTerm b=lastLogIndex
                               RVResp: a=voteGranted
                               AEReq: a=prevLogIndex b=prevLogTerm c=commitIndex d=#entries
                               AEResp: a=success b=matchIndex */
    uint8_t et, ev, pad0, pad1;   /* AEReq entry (term, value) when d == 1 */
    uint32_t pad2;
    Log mlog;               /* RVResp, AEReq */
} Msg;

typedef struct {
    uint8_t term, leader, votes, vlp;  /* vlp: domain of evoterLog (bitmask) */
    uint32_t pad;
    Log elog;
    Log vl[NMAX];
} Elec;

typedef struct {
    uint8_t term, role, voted, commit, vresp, vgrant, vlp, pad;
    Log log;
    Log vl[NMAX];
    uint8_t next[NMAX], match[NMAX];
    uint8_t pad2[6];
} Srv;

typedef struct {
    int nmsg, nelec, nall, pad;
    Msg msg[KMAX];
    uint8_t cnt[KMAX];
    Elec elec[EMAX];
    Log all[AMAX];
    Srv s[NMAX];
} State;

typedef struct {
    orc_cfg c;
} Ctx;

/* ------------------------------------------------------------ ordering -- */
static int msg_cmp(const Msg *x, const Msg *y) { return memcmp(x, y, sizeof(Msg)); }
static int elec_cmp(const Elec *x, const Elec *y) { return memcmp(x, y, sizeof(Elec)); }

static void state_copy(State *d, const State *s) {
    d->nmsg = s->nmsg; d->nelec = s->nelec; d->nall = s->nall;
    memcpy(d->msg, s->msg, sizeof(Msg) * s->nmsg);
    memcpy(d->cnt, s->cnt, s->nmsg);
    memcpy(d->elec, s->elec, sizeof(Elec) * s->nelec);
    memcpy(d->all, s->all, sizeof(Log) * s->nall);
    memcpy(d->s, s->s, sizeof(d->s));
}

static int g_overflow;  /* set on any capacity overflow: a hard error */

static int bag_find(const State *s, const Msg *m, int *pos) {
    int lo = 0, hi = s->nmsg;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        int c = msg_cmp(&s->msg[mid], m);
        if (c == 0) { *pos = mid; return 1; }
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    *pos = lo;
    return 0;
}

/* raft.tla:106-110 WithMessage */
static void with_message(State *s, const Msg *m) {
    int p;
    if (bag_find(s, m, &p)) { s->cnt[p]++; return; }
    if (s->nmsg >= KMAX) { g_overflow = 1; return; }
    memmove(&s->msg[p + 1], &s->msg[p], sizeof(Msg) * (s->nmsg - p));
    memmove(&s->cnt[p + 1], &s->cnt[p], s->nmsg - p);
    s->msg[p] = *m; s->cnt[p] = 1; s->nmsg++;
}

/* raft.tla:114-119 WithoutMessage */
static void without_message(State *s, const Msg *m) {
    int p;
    if (!bag_find(s, m, &p)) return;
    if (s->cnt[p] <= 1) {
        memmove(&s->msg[p], &s->msg[p + 1], sizeof(Msg) * (s->nmsg - p - 1));
        memmove(&s->cnt[p], &s->cnt[p + 1], s->nmsg - p - 1);
        s->nmsg--;
    } else {
        s->cnt[p]--;
    }
}

static void all_add(State *s, Log l) {
    int lo = 0, hi = s->nall;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (s->all[mid] == l) return;
        if (s->all[mid] < l) lo = mid + 1; else hi = mid;
    }
    if (s->nall >= AMAX) { g_overflow = 1; return; }
    memmove(&s->all[lo + 1], &s->all[lo], sizeof(Log) * (s->nall - lo));
    s->all[lo] = l; s->nall++;
}

static void elec_add(State *s, const Elec *e) {
    int lo = 0, hi = s->nelec;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        int c = elec_cmp(&s->elec[mid], e);
        if (c == 0) return;
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    if (s->nelec >= EMAX) { g_overflow = 1; return; }
    memmove(&s->elec[lo + 1], &s->elec[lo], sizeof(Elec) * (s->nelec - lo));
    s->elec[lo] = *e; s->nelec++;
}

/* ---------------------------------------------------------------- init -- */
/* raft.tla:140-160 */
static void init_state(const orc_cfg *c, State *s) {
    memset(s, 0, sizeof(*s));
    for (int i = 0; i < c->n_server; i++) {
        Srv *v = &s->s[i];
        v->term = 1; v->role = FOLLOWER; v->voted = NIL;
        for (int j = 0; j < c->n_server; j++) { v->next[j] = 1; v->match[j] = 0; }
    }
}

/* ------------------------------------------------------------- actions -- */
typedef void (*emit_fn)(void *ud, const State *succ, int action, int arg);

enum {
    A_RESTART = 0, A_TIMEOUT, A_REQUESTVOTE, A_BECOMELEADER, A_CLIENTREQUEST,
    A_ADVANCECOMMIT, A_APPENDENTRIES, A_UPDATETERM, A_HRVREQ, A_HRVRESP,
    A_HAEREQ, A_HAERESP, A_DROPSTALE, A_DUPLICATE, A_DROP, A_COUNT
};
static const char *ACTION_NAME[A_COUNT] = {
    "Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
    "AdvanceCommitIndex", "AppendEntries", "UpdateTerm", "HandleRequestVoteRequest",
    "HandleRequestVoteResponse", "HandleAppendEntriesRequest",
    "HandleAppendEntriesResponse", "DropStaleResponse", "DuplicateMessage", "DropMessage"};

static int g_spec_error;  /* TLC evaluation error (index out of domain) */

static int log_term_checked(Log l, int k) {
    if (k < 1 || k > log_len(l)) { g_spec_error = 1; return 0; }
    return log_term(l, k);
}

/* Expand all enabled instances of Next (raft.tla:454-465).  `tmp` is scratch.
 * allLogs' = allLogs \cup {log[i]} (pre-state logs, :465) is applied to
 * every successor by the caller-supplied `base`. */
static void expand(const orc_cfg *c, const State *s, State *base, State *t, emit_fn emit, void *ud) {
    const int N = c->n_server;
    /* base: s with allLogs' applied (:465) */
    state_copy(base, s);
    for (int i = 0; i < N; i++) all_add(base, s->s[i].log);

#define BEGIN() state_copy(t, base)
    /* Restart(i)  :167-175 */
    for (int i = 0; i < N; i++) {
        BEGIN();
        Srv *v = &t->s[i];
        v->role = FOLLOWER; v->vresp = 0; v->vgrant = 0; v->vlp = 0;
        memset(v->vl, 0, sizeof(v->vl));
        for (int j = 0; j < N; j++) { v->next[j] = 1; v->match[j] = 0; }
        v->commit = 0;
        emit(ud, t, A_RESTART, i);
    }
    /* Timeout(i)  :178-187 */
    for (int i = 0; i < N; i++) {
        const Srv *u = &s->s[i];
        if (u->role != FOLLOWER && u->role != CANDIDATE) continue;
        BEGIN();
        Srv *v = &t->s[i];
        v->role = CANDIDATE; v->term = u->term + 1; v->voted = NIL;
        v->vresp = 0; v->vgrant = 0; v->vlp = 0; memset(v->vl, 0, sizeof(v->vl));
        emit(ud, t, A_TIMEOUT, i);
    }
    /* RequestVote(i, j)  :190-199 */
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) {
            const Srv *u = &s->s[i];
            if (u->role != CANDIDATE || (u->vresp >> j & 1)) continue;
            BEGIN();
            Msg m; memset(&m, 0, sizeof m);
            m.type = RVREQ; m.term = u->term; m.a = (uint8_t)last_term(u->log);
            m.b = (uint8_t)log_len(u->log); m.src = (uint8_t)i; m.dst = (uint8_t)j;
            with_message(t, &m);
            emit(ud, t, A_REQUESTVOTE, i * 8 + j);
        }
    /* BecomeLeader(i)  :229-243 */
    for (int i = 0; i < N; i++) {
        const Srv *u = &s->s[i];
        if (u->role != CANDIDATE || !(__builtin_popcount(u->vgrant) * 2 > N)) continue;
        BEGIN();
        Srv *v = &t->s[i];
        v->role = LEADER;
        for (int j = 0; j < N; j++) { v->next[j] = (uint8_t)(log_len(u->log) + 1); v->match[j] = 0; }
        Elec e; memset(&e, 0, sizeof e);
        e.term = u->term; e.leader = (uint8_t)i; e.elog = u->log; e.votes = u->vgrant;
        e.vlp = u->vlp;
        for (int j = 0; j < N; j++) if (u->vlp >> j & 1) e.vl[j] = u->vl[j];
        elec_add(t, &e);
        emit(ud, t, A_BECOMELEADER, i);
    }
    /* ClientRequest(i, v)  :246-253 */
    for (int i = 0; i < N; i++)
        for (int val = 0; val < c->n_value; val++) {
            const Srv *u = &s->s[i];
            if (u->role != LEADER) continue;
            if (log_len(u->log) >= LCAP) { g_overflow = 1; continue; }
            BEGIN();
            t->s[i].log = log_append(u->log, u->term, val);
            emit(ud, t, A_CLIENTREQUEST, i * 8 + val);
        }
    /* AdvanceCommitIndex(i)  :259-276 */
    for (int i = 0; i < N; i++) {
        const Srv *u = &s->s[i];
        if (u->role != LEADER) continue;
        int maxagree = 0;
        for (int index = 1; index <= log_len(u->log); index++) {
            int agree = 1;   /* {i} */
            for (int k = 0; k < N; k++) if (k != i && u->match[k] >= index) agree++;
            if (agree * 2 > N) maxagree = index;
        }
        int nci = u->commit;
        if (maxagree > 0 && log_term_checked(u->log, maxagree) == u->term) nci = maxagree;
        BEGIN();
        t->s[i].commit = (uint8_t)nci;
        emit(ud, t, A_ADVANCECOMMIT, i);
    }
    /* AppendEntries(i, j)  :204-226 */
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) {
            const Srv *u = &s->s[i];
            if (i == j || u->role != LEADER) continue;
            int nxt = u->next[j];
            int prev = nxt - 1;
            int prevt = prev > 0 ? log_term_checked(u->log, prev) : 0;
            int len = log_len(u->log);
            int last = len < nxt ? len : nxt;
            BEGIN();
            Msg m; memset(&m, 0, sizeof m);
            m.type = AEREQ; m.term = u->term; m.a = (uint8_t)prev; m.b = (uint8_t)prevt;
            if (nxt <= last) { m.d = 1; m.et = (uint8_t)log_term(u->log, nxt); m.ev = (uint8_t)log_val(u->log, nxt); }
            m.mlog = u->log;
            m.c = (uint8_t)(u->commit < last ? u->commit : last);
            m.src = (uint8_t)i; m.dst = (uint8_t)j;
            with_message(t, &m);
            emit(ud, t, A_APPENDENTRIES, i * 8 + j);
        }
    /* \E m \in DOMAIN messages : Receive(m)  :421-436 */
    for (int k = 0; k < s->nmsg; k++) {
        const Msg *m = &s->msg[k];
        const int i = m->dst, j = m->src;
        const Srv *u = &s->s[i];
        if (m->term > u->term) {            /* UpdateTerm :406-412 */
            BEGIN();
            Srv *v = &t->s[i];
            v->term = m->term; v->role = FOLLOWER; v->voted = NIL;
            emit(ud, t, A_UPDATETERM, k);
            continue;
        }
        if (m->type == RVREQ) {             /* HandleRequestVoteRequest :284-303 */
            int lt = last_term(u->log);
            int logok = m->a > lt || (m->a == lt && m->b >= log_len(u->log));
            int grant = m->term == u->term && logok && (u->voted == NIL || u->voted == j);
            BEGIN();
            if (grant) t->s[i].voted = (uint8_t)j;
            Msg r; memset(&r, 0, sizeof r);
            r.type = RVRESP; r.term = u->term; r.a = (uint8_t)grant; r.mlog = u->log;
            r.src = (uint8_t)i; r.dst = (uint8_t)j;
            with_message(t, &r);      /* Reply: add the response first ... */
            without_message(t, m);    /* ... then remove the request :129-130 */
            emit(ud, t, A_HRVREQ, k);
        } else if (m->type == RVRESP || m->type == AERESP) {
            if (m->term < u->term) {        /* DropStaleResponse :415-418 */
                BEGIN();
                without_message(t, m);
                emit(ud, t, A_DROPSTALE, k);
            } else if (m->type == RVRESP) { /* HandleRequestVoteResponse :307-321 */
                BEGIN();
                Srv *v = &t->s[i];
                v->vresp |= (uint8_t)(1 << j);
                if (m->a) {
                    v->vgrant |= (uint8_t)(1 << j);
                    if (!(v->vlp >> j & 1)) { v->vlp |= (uint8_t)(1 << j); v->vl[j] = m->mlog; }  /* @@ keeps left */
                }
                without_message(t, m);
                emit(ud, t, A_HRVRESP, k);
            } else {                        /* HandleAppendEntriesResponse :393-403 */
                BEGIN();
                Srv *v = &t->s[i];
                if (m->a) { v->next[j] = (uint8_t)(m->b + 1); v->match[j] = m->b; }
                else { int nx = u->next[j] - 1; v->next[j] = (uint8_t)(nx > 1 ? nx : 1); }
                without_message(t, m);
                emit(ud, t, A_HAERESP, k);
            }
        } else {                            /* HandleAppendEntriesRequest :327-389 */
            int len = log_len(u->log);
            int logok = m->a == 0 || (m->a > 0 && m->a <= len && m->b == log_term(u->log, m->a));
            if (m->term < u->term || (m->term == u->term && u->role == FOLLOWER && !logok)) {
                BEGIN();                    /* reject :333-345 */
                Msg r; memset(&r, 0, sizeof r);
                r.type = AERESP; r.term = u->term; r.a = 0; r.b = 0;
                r.src = (uint8_t)i; r.dst = (uint8_t)j;
                with_message(t, &r);
                without_message(t, m);
                emit(ud, t, A_HAEREQ, k);
            } else if (m->term == u->term && u->role == CANDIDATE) {
                BEGIN();                    /* return to follower :346-350 */
                t->s[i].role = FOLLOWER;
                emit(ud, t, A_HAEREQ, k);
            } else if (m->term == u->term && u->role == FOLLOWER && logok) {
                int index = m->a + 1;       /* accept :351-388 */
                if (m->d == 0 || (len >= index && log_term(u->log, index) == m->et)) {
                    BEGIN();                /* already done :356-374 */
                    t->s[i].commit = m->c;
                    Msg r; memset(&r, 0, sizeof r);
                    r.type = AERESP; r.term = u->term; r.a = 1; r.b = (uint8_t)(m->a + m->d);
                    r.src = (uint8_t)i; r.dst = (uint8_t)j;
                    with_message(t, &r);
                    without_message(t, m);
                    emit(ud, t, A_HAEREQ, k);
                } else if (len >= index) {  /* conflict: remove 1 entry :375-382 */
                    BEGIN();
                    t->s[i].log = log_prefix(u->log, len - 1);
                    emit(ud, t, A_HAEREQ, k);
                } else if (len == m->a) {   /* no conflict: append :383-388 */
                    BEGIN();
                    t->s[i].log = log_append(u->log, m->et, m->ev);
                    emit(ud, t, A_HAEREQ, k);
                }
            }
            /* AEReq at equal term to a Leader: no disjunct enabled */
        }
    }
    /* DuplicateMessage(m) :443-445 */
    for (int k = 0; k < s->nmsg; k++) {
        BEGIN();
        t->cnt[k]++;     /* same key, count + 1 */
        emit(ud, t, A_DUPLICATE, k);
    }
    /* DropMessage(m) :448-450 */
    for (int k = 0; k < s->nmsg; k++) {
        BEGIN();
        without_message(t, &s->msg[k]);
        emit(ud, t, A_DROP, k);
    }
#undef BEGIN
}

/* ------------------------------------------------ MC wrapper (MC.tla) -- */
static int in_model(const orc_cfg *c, const State *s) {
    for (int i = 0; i < c->n_server; i++) {
        if (s->s[i].term > c->max_term) return 0;
        if (log_len(s->s[i].log) > c->max_log) return 0;
    }
    int total = 0;
    for (int k = 0; k < s->nmsg; k++) { if (s->cnt[k] > c->max_copies) return 0; total += s->cnt[k]; }
    if (c->max_msgs && total > c->max_msgs) return 0;
    return 1;
}

/* returns bitmask of VIOLATED invariants among c->inv_mask */
static int check_inv(const orc_cfg *c, const State *s) {
    int bad = 0;
    const int N = c->n_server;
    if (c->inv_mask & ORC_INV_NO_TWO_LEADERS) {
        int nl = 0;
        for (int i = 0; i < N; i++) nl += s->s[i].role == LEADER;
        if (nl > 1) bad |= ORC_INV_NO_TWO_LEADERS;
    }
    if (c->inv_mask & ORC_INV_ELECTION_SAFETY) {
        for (int a = 0; a < s->nelec; a++)
            for (int b = 0; b < s->nelec; b++)
                if (s->elec[a].term == s->elec[b].term && s->elec[a].leader != s->elec[b].leader)
                    bad |= ORC_INV_ELECTION_SAFETY;
    }
    if (c->inv_mask & ORC_INV_LOG_MATCHING) {
        for (int i = 0; i < N; i++)
            for (int j = 0; j < N; j++) {
                Log a = s->s[i].log, b = s->s[j].log;
                int m = log_len(a) < log_len(b) ? log_len(a) : log_len(b);
                for (int n = 1; n <= m; n++)
                    if (log_term(a, n) == log_term(b, n) && log_prefix(a, n) != log_prefix(b, n))
                        bad |= ORC_INV_LOG_MATCHING;
            }
    }
    return bad;
}

/* --------------------------------------------- canonical serialisation -- */
/* Injective compact byte encoding of a canonical State. */
static inline uint8_t *put_log(uint8_t *p, Log l) {
    int n = log_len(l);
    *p++ = (uint8_t)n;
    for (int k = 1; k <= n; k++) *p++ = (uint8_t)((log_term(l, k) << 4) | log_val(l, k));
    return p;
}
static inline const uint8_t *get_log(const uint8_t *p, Log *l) {
    int n = *p++;
    Log x = 0;
    for (int k = 0; k < n; k++) { int e = *p++; x = log_append(x, e >> 4, e & 15); }
    *l = x;
    return p;
}

static size_t serialize(const orc_cfg *c, const State *s, uint8_t *out) {
    uint8_t *p = out;
    const int N = c->n_server;
    *p++ = (uint8_t)s->nmsg;
    for (int k = 0; k < s->nmsg; k++) {
        const Msg *m = &s->msg[k];
        *p++ = m->type; *p++ = m->term; *p++ = (uint8_t)(m->src << 4 | m->dst);
        *p++ = m->a; *p++ = m->b; *p++ = m->c; *p++ = m->d; *p++ = m->et; *p++ = m->ev;
        if (m->type == RVRESP || m->type == AEREQ) p = put_log(p, m->mlog);
        *p++ = s->cnt[k];
    }
    *p++ = (uint8_t)s->nelec;
    for (int k = 0; k < s->nelec; k++) {
        const Elec *e = &s->elec[k];
        *p++ = e->term; *p++ = e->leader; *p++ = e->votes; *p++ = e->vlp;
        p = put_log(p, e->elog);
        for (int j = 0; j < N; j++) if (e->vlp >> j & 1) p = put_log(p, e->vl[j]);
    }
    *p++ = (uint8_t)(s->nall & 255); *p++ = (uint8_t)(s->nall >> 8);
    for (int k = 0; k < s->nall; k++) p = put_log(p, s->all[k]);
    for (int i = 0; i < N; i++) {
        const Srv *v = &s->s[i];
        *p++ = v->term; *p++ = v->role; *p++ = v->voted; *p++ = v->commit;
        *p++ = v->vresp; *p++ = v->vgrant; *p++ = v->vlp;
        p = put_log(p, v->log);
        for (int j = 0; j < N; j++) if (v->vlp >> j & 1) p = put_log(p, v->vl[j]);
        for (int j = 0; j < N; j++) { *p++ = v->next[j]; *p++ = v->match[j]; }
    }
    return (size_t)(p - out);
}

static void deserialize(const orc_cfg *c, const uint8_t *p, State *s) {
    const int N = c->n_server;
    s->nmsg = *p++;
    for (int k = 0; k < s->nmsg; k++) {
        Msg *m = &s->msg[k];
        memset(m, 0, sizeof *m);
        m->type = *p++; m->term = *p++; m->src = *p >> 4; m->dst = *p & 15; p++;
        m->a = *p++; m->b = *p++; m->c = *p++; m->d = *p++; m->et = *p++; m->ev = *p++;
        if (m->type == RVRESP || m->type == AEREQ) p = get_log(p, &m->mlog);
        s->cnt[k] = *p++;
    }
    s->nelec = *p++;
    for (int k = 0; k < s->nelec; k++) {
        Elec *e = &s->elec[k];
        memset(e, 0, sizeof *e);
        e->term = *p++; e->leader = *p++; e->votes = *p++; e->vlp = *p++;
        p = get_log(p, &e->elog);
        for (int j = 0; j < N; j++) if (e->vlp >> j & 1) p = get_log(p, &e->vl[j]);
    }
    s->nall = p[0] | (p[1] << 8); p += 2;
    for (int k = 0; k < s->nall; k++) p = get_log(p, &s->all[k]);
    for (int i = 0; i < N; i++) {
        Srv *v = &s->s[i];
        memset(v, 0, sizeof *v);
        v->term = *p++; v->role = *p++; v->voted = *p++; v->commit = *p++;
        v->vresp = *p++; v->vgrant = *p++; v->vlp = *p++;
        p = get_log(p, &v->log);
        for (int j = 0; j < N; j++) if (v->vlp >> j & 1) p = get_log(p, &v->vl[j]);
        for (int j = 0; j < N; j++) { v->next[j] = *p++; v->match[j] = *p++; }
    }
}

/* 128-bit hash of bytes (two independent 64-bit multiply-xorshift lanes). */
static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32; x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32;
    return x;
}
static void hash128(const uint8_t *p, size_t n, uint64_t *h1, uint64_t *h2) {
    uint64_t a = 0x243f6a8885a308d3ULL ^ n, b = 0x13198a2e03707344ULL ^ (n * 0x9E3779B97F4A7C15ULL);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w; memcpy(&w, p + i, 8);
        a = mix64(a ^ w) + 0x9E3779B97F4A7C15ULL;
        b = mix64(b + w * 0xff51afd7ed558ccdULL) ^ 0xc4ceb9fe1a85ec53ULL;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    a = mix64(a ^ w ^ 0xa0761d6478bd642fULL);
    b = mix64(b + w * 0xe7037ed1a0b428dbULL + 1);
    *h1 = a; *h2 = b | 1;   /* h2 != 0 marks an occupied slot */
}

/* ----------------------------------------------------------- symmetry -- */
/* SYMMETRY Permutations(Server) (specs/MC.tla): TLC identifies a state with
 * its server-permuted images.  The oracle's orbit key is the
 * lexicographically least serialisation over all N! permutations pi, where
 * pi relabels every server-valued field (votedFor, the vote sets, the
 * voterLog and next/matchIndex domains, msource/mdest, eleader, evotes,
 * evoterLog) and moves server record i to pi(i); bag and elections are
 * re-sorted.  Any exact orbit invariant gives the same counts. */
static uint8_t perm_mask(uint8_t m, const int *pi, int N) {
    uint8_t r = 0;
    for (int j = 0; j < N; j++) if (m >> j & 1) r |= (uint8_t)(1 << pi[j]);
    return r;
}
static int cmp_msg_cnt(const void *a, const void *b) { return msg_cmp((const Msg *)a, (const Msg *)b); }
static void permute_state(const orc_cfg *c, const State *s, const int *pi, State *o) {
    const int N = c->n_server;
    state_copy(o, s);
    for (int i = 0; i < N; i++) {
        const Srv *v = &s->s[i];
        Srv *w = &o->s[pi[i]];
        *w = *v;
        w->voted = v->voted == NIL ? NIL : (uint8_t)pi[v->voted];
        w->vresp = perm_mask(v->vresp, pi, N); w->vgrant = perm_mask(v->vgrant, pi, N);
        w->vlp = perm_mask(v->vlp, pi, N);
        for (int j = 0; j < N; j++) { w->vl[pi[j]] = v->vl[j]; w->next[pi[j]] = v->next[j]; w->match[pi[j]] = v->match[j]; }
    }
    /* bag: relabel, then sort (msg, cnt) pairs by message */
    struct { Msg m; uint8_t cnt; } tmp[KMAX];
    for (int k = 0; k < s->nmsg; k++) {
        tmp[k].m = s->msg[k];
        tmp[k].m.src = (uint8_t)pi[s->msg[k].src]; tmp[k].m.dst = (uint8_t)pi[s->msg[k].dst];
        tmp[k].cnt = s->cnt[k];
    }
    qsort(tmp, (size_t)s->nmsg, sizeof tmp[0], cmp_msg_cnt);
    for (int k = 0; k < s->nmsg; k++) { o->msg[k] = tmp[k].m; o->cnt[k] = tmp[k].cnt; }
    for (int k = 0; k < s->nelec; k++) {
        const Elec *e = &s->elec[k];
        Elec *f = &o->elec[k];
        *f = *e;
        f->leader = (uint8_t)pi[e->leader]; f->votes = perm_mask(e->votes, pi, N); f->vlp = perm_mask(e->vlp, pi, N);
        for (int j = 0; j < N; j++) f->vl[pi[j]] = e->vl[j];
    }
    qsort(o->elec, (size_t)s->nelec, sizeof(Elec), (int (*)(const void *, const void *))elec_cmp);
}
/* next permutation of pi[0..N) in lexicographic order; 0 after the last */
static int next_perm(int *pi, int N) {
    int i = N - 2;
    while (i >= 0 && pi[i] > pi[i + 1]) i--;
    if (i < 0) return 0;
    int j = N - 1;
    while (pi[j] < pi[i]) j--;
    int t = pi[i]; pi[i] = pi[j]; pi[j] = t;
    for (int a = i + 1, b2 = N - 1; a < b2; a++, b2--) { t = pi[a]; pi[a] = pi[b2]; pi[b2] = t; }
    return 1;
}

/* Orbit serialisation of the image pi(s): an injective byte encoding of the
 * permuted state with the server fields FIRST, field-major (the N terms in
 * position order -- position p holds server sigma[p] = pi^-1(p) -- then the
 * N roles, then every relabelled field: votedFor, commitIndex, the vote
 * sets, voterLog domain, log, nextIndex / matchIndex, voterLog), then the
 * relabelled bag and elections re-sorted, then allLogs.  With `best` set,
 * the bytes are compared with best's as they are produced: the image is
 * dropped (returns 1) at its first byte above best's, returns 0 if it equals
 * best, -1 if it is smaller (then the whole image is in out). */
static int ser_image(const orc_cfg *c, const State *s, const int *pi, const int *sigma, uint8_t *out,
                     const uint8_t *best) {
    const int N = c->n_server;
    int st = best ? 0 : -1;     /* 0: equal to best so far; -1: below best (or no best): write on */
    size_t n = 0;
#define PUT(b_)                                                             \
    do {                                                                    \
        const uint8_t v_ = (uint8_t)(b_);                                   \
        if (st == 0) { if (v_ > best[n]) return 1; if (v_ < best[n]) st = -1; } \
        out[n++] = v_;                                                      \
    } while (0)
#define PUTLOG(l_)                                                          \
    do {                                                                    \
        const Log L_ = (l_); const int k_ = log_len(L_);                    \
        PUT(k_);                                                            \
        for (int e_ = 1; e_ <= k_; e_++) PUT((log_term(L_, e_) << 4) | log_val(L_, e_)); \
    } while (0)
    for (int p = 0; p < N; p++) PUT(s->s[sigma[p]].term);
    for (int p = 0; p < N; p++) PUT(s->s[sigma[p]].role);
    for (int p = 0; p < N; p++) {
        const Srv *v = &s->s[sigma[p]];
        PUT(v->voted == NIL ? NIL : pi[v->voted]); PUT(v->commit);
        PUT(perm_mask(v->vresp, pi, N)); PUT(perm_mask(v->vgrant, pi, N));
        const uint8_t vlp = perm_mask(v->vlp, pi, N);
        PUT(vlp);
        PUTLOG(v->log);
        for (int q = 0; q < N; q++) { PUT(v->next[sigma[q]]); PUT(v->match[sigma[q]]); }
        for (int q = 0; q < N; q++) if (vlp >> q & 1) PUTLOG(v->vl[sigma[q]]);
    }
    /* bag: relabel, re-sort */
    struct { Msg m; uint8_t cnt; } bag[KMAX];
    for (int k = 0; k < s->nmsg; k++) {
        bag[k].m = s->msg[k];
        bag[k].m.src = (uint8_t)pi[s->msg[k].src]; bag[k].m.dst = (uint8_t)pi[s->msg[k].dst];
        bag[k].cnt = s->cnt[k];
    }
    qsort(bag, (size_t)s->nmsg, sizeof bag[0], cmp_msg_cnt);
    PUT(s->nmsg);
    for (int k = 0; k < s->nmsg; k++) {
        const Msg *m = &bag[k].m;
        PUT(m->type); PUT(m->term); PUT(m->src << 4 | m->dst);
        PUT(m->a); PUT(m->b); PUT(m->c); PUT(m->d); PUT(m->et); PUT(m->ev);
        if (m->type == RVRESP || m->type == AEREQ) PUTLOG(m->mlog);
        PUT(bag[k].cnt);
    }
    Elec el[EMAX];
    for (int k = 0; k < s->nelec; k++) {
        const Elec *e = &s->elec[k];
        Elec *f = &el[k];
        *f = *e;
        f->leader = (uint8_t)pi[e->leader]; f->votes = perm_mask(e->votes, pi, N); f->vlp = perm_mask(e->vlp, pi, N);
        memset(f->vl, 0, sizeof f->vl);
        for (int j = 0; j < N; j++) f->vl[pi[j]] = e->vl[j];
    }
    qsort(el, (size_t)s->nelec, sizeof(Elec), (int (*)(const void *, const void *))elec_cmp);
    PUT(s->nelec);
    for (int k = 0; k < s->nelec; k++) {
        const Elec *e = &el[k];
        PUT(e->term); PUT(e->leader); PUT(e->votes); PUT(e->vlp);
        PUTLOG(e->elog);
        for (int j = 0; j < N; j++) if (e->vlp >> j & 1) PUTLOG(e->vl[j]);
    }
    PUT(s->nall & 255); PUT(s->nall >> 8);
    for (int k = 0; k < s->nall; k++) PUTLOG(s->all[k]);
#undef PUTLOG
#undef PUT
    return st;
}

/* Orderings sigma (position -> server) of the servers sorted by key[],
 * permuting only within ties: sg_first starts them, sg_next advances (0
 * after the last).  gb[0..ng] bound the tie groups. */
static int sg_first(const int *key, int N, int *sg, int *gb) {
    for (int i = 0; i < N; i++) sg[i] = i;
    for (int i = 1; i < N; i++)       /* stable insertion sort by key */
        for (int j = i; j > 0 && key[sg[j - 1]] > key[sg[j]]; j--) { int t = sg[j]; sg[j] = sg[j - 1]; sg[j - 1] = t; }
    int ng = 0;
    for (int p = 0; p < N; p++) if (!p || key[sg[p]] != key[sg[p - 1]]) gb[ng++] = p;
    gb[ng] = N;
    return ng;
}
static int sg_next(int *sg, const int *gb, int ng) {
    int g = ng - 1;   /* an odometer over the tie groups' permutations */
    while (g >= 0 && !next_perm(sg + gb[g], gb[g + 1] - gb[g])) {
        /* (the group is in its last, descending order: back to ascending) */
        for (int a = gb[g], b2 = gb[g + 1] - 1; a < b2; a++, b2--) { int t = sg[a]; sg[a] = sg[b2]; sg[b2] = t; }
        g--;
    }
    return g >= 0;
}

/* serialise the orbit representative of s (the least orbit serialisation
 * over all N! images) into out; returns its length.  Without SYMMETRY: the
 * plain serialisation.  The least image begins with the N terms in
 * ascending order, then within equal terms the roles ascending: every other
 * image is above it in those first 2N bytes, so only the orderings of the
 * servers tied on (term, role) are serialised and compared. */
static size_t serialize_canon(const orc_cfg *c, const State *s, uint8_t *out) {
    const int N = c->n_server;
    if (!c->symmetry) return serialize(c, s, out);
    int key[NMAX] = {0}, sg[NMAX], gb[NMAX + 1], pi[NMAX];
    for (int i = 0; i < N; i++) key[i] = s->s[i].term * 4 + s->s[i].role;
    const int ng = sg_first(key, N, sg, gb);
    static __thread uint8_t *scratch;   /* per worker thread, never freed */
    if (!scratch) scratch = (uint8_t *)malloc(1 << 17);
    uint8_t *tmp = scratch, *best = out;
    const size_t len = serialize(c, s, tmp);   /* the orbit serialisation has the same length */
    int first = 1;
    do {
        for (int p = 0; p < N; p++) pi[sg[p]] = p;
        if (ser_image(c, s, pi, sg, first ? best : tmp, first ? NULL : best) < 0 && !first) {
            uint8_t *t = best; best = tmp; tmp = t;
        }
        first = 0;
    } while (sg_next(sg, gb, ng));
    if (best != out) memcpy(out, best, len);
    return len;
}

/* ------------------------------------------------------ orbit text digest -- */
/* The digest of a SYMMETRY level is the sum of FNV-1a-64 of each orbit's
 * ORBIT TEXT: the TLC text (state_text below) of the image pi(s) whose
 * "rotated text" is least over all N! permutations, where the rotated text is
 * the state text with its three lines that name no server function
 * (messages, elections, allLogs) moved after the ten per-server lines.  It
 * is a function of the orbit alone and is defined on TLC value text, so the
 * product (rtla_level_orbit_hash, over its packed rows) and the value oracle
 * (raft_values.orbit_text) compute it independently.  Here the per-server
 * lines of each image are rendered with an early exit against the best so
 * far; only images tying with it through them render their bag and elections. */
typedef struct { char *p; size_t n; const char *best; size_t bn; int st; } RText;
/* append t[0..k) comparing with best; returns 1 when the image is above best */
static inline int rt_put(RText *r, const char *t, size_t k) {
    if (r->st == 0) {
        const size_t m = k < r->bn - r->n ? k : r->bn - r->n;
        const int d = memcmp(t, r->best + r->n, m);
        if (d > 0 || (d == 0 && m < k)) return 1;   /* (m < k: best ended first -- cannot happen) */
        if (d < 0) r->st = -1;
    }
    memcpy(r->p + r->n, t, k);
    r->n += k;
    return 0;
}
static inline int rt_s(RText *r, const char *t) { return rt_put(r, t, strlen(t)); }
static inline int rt_u(RText *r, unsigned v) {
    char b[12]; int k = 0; char t[12];
    do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    for (int i = 0; i < k; i++) b[i] = t[k - 1 - i];
    return rt_put(r, b, (size_t)k);
}
static inline int rt_srv(RText *r, int j) { char b[3] = {'s', (char)('1' + j), 0}; return rt_put(r, b, 2); }
static int rt_log(RText *r, Log l) {
    const int n = log_len(l);
    if (!n) return rt_s(r, "<<>>");
    if (rt_s(r, "<<")) return 1;
    for (int k = 1; k <= n; k++) {
        if (k > 1 && rt_s(r, ", ")) return 1;
        if (rt_s(r, "[term |-> ") || rt_u(r, (unsigned)log_term(l, k)) || rt_s(r, ", value |-> v") ||
            rt_u(r, (unsigned)log_val(l, k) + 1) || rt_s(r, "]"))
            return 1;
    }
    return rt_s(r, ">>");
}
static int rt_srvset(RText *r, int mask, int N) {
    if (rt_s(r, "{")) return 1;
    int first = 1;
    for (int j = 0; j < N; j++)
        if (mask >> j & 1) { if ((!first && rt_s(r, ", ")) || rt_srv(r, j)) return 1; first = 0; }
    return rt_s(r, "}");
}
/* the per-server lines [from, 10) of the image pi(s) (sigma = pi^-1), each starting "\n" */
static int rt_servers(const orc_cfg *c, const State *s, const int *pi, const int *sigma, RText *r, int from) {
    const int N = c->n_server;
    static const char *RN[3] = {"\"Follower\"", "\"Candidate\"", "\"Leader\""};
    int ln = 0;
#define LINE(name, body)                                                        \
    if (ln++ >= from) {                                                         \
        if (rt_s(r, "\n/\\ " name " = (")) return 1;                            \
        for (int p = 0; p < N; p++) {                                           \
            const Srv *v = &s->s[sigma[p]]; (void)v;                            \
            if ((p && rt_s(r, " @@ ")) || rt_srv(r, p) || rt_s(r, " :> ")) return 1; \
            body;                                                               \
        }                                                                       \
        if (rt_s(r, ")")) return 1;                                             \
    }
    LINE("currentTerm", if (rt_u(r, v->term)) return 1);
    LINE("state", if (rt_s(r, RN[v->role])) return 1);
    LINE("votedFor", if (v->voted == NIL ? rt_s(r, "\"Nil\"") : rt_srv(r, pi[v->voted])) return 1);
    LINE("log", if (rt_log(r, v->log)) return 1);
    LINE("commitIndex", if (rt_u(r, v->commit)) return 1);
    LINE("votesResponded", if (rt_srvset(r, perm_mask(v->vresp, pi, N), N)) return 1);
    LINE("votesGranted", if (rt_srvset(r, perm_mask(v->vgrant, pi, N), N)) return 1);
    LINE("voterLog", {
        const int vlp = perm_mask(v->vlp, pi, N);
        if (!vlp) { if (rt_s(r, "<<>>")) return 1; }
        else {
            if (rt_s(r, "(")) return 1;
            int first = 1;
            for (int q = 0; q < N; q++)
                if (vlp >> q & 1) {
                    if ((!first && rt_s(r, " @@ ")) || rt_srv(r, q) || rt_s(r, " :> ") || rt_log(r, v->vl[sigma[q]]))
                        return 1;
                    first = 0;
                }
            if (rt_s(r, ")")) return 1;
        }
    });
    LINE("nextIndex", {
        if (rt_s(r, "(")) return 1;
        for (int q = 0; q < N; q++)
            if ((q && rt_s(r, " @@ ")) || rt_srv(r, q) || rt_s(r, " :> ") || rt_u(r, v->next[sigma[q]])) return 1;
        if (rt_s(r, ")")) return 1;
    });
    LINE("matchIndex", {
        if (rt_s(r, "(")) return 1;
        for (int q = 0; q < N; q++)
            if ((q && rt_s(r, " @@ ")) || rt_srv(r, q) || rt_s(r, " :> ") || rt_u(r, v->match[sigma[q]])) return 1;
        if (rt_s(r, ")")) return 1;
    });
#undef LINE
    return 0;
}
/* One message item "<record> :> count" of the image pi(s). */
static void rt_msg(RText *r, const Msg *m, int cnt, const int *pi) {
    static const char *TN[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                                "AppendEntriesResponse"};
    rt_s(r, "[mtype |-> \""); rt_s(r, TN[m->type]); rt_s(r, "\", mterm |-> "); rt_u(r, m->term); rt_s(r, ", ");
    switch (m->type) {
    case RVREQ:
        rt_s(r, "mlastLogTerm |-> "); rt_u(r, m->a); rt_s(r, ", mlastLogIndex |-> "); rt_u(r, m->b); rt_s(r, ", ");
        break;
    case RVRESP:
        rt_s(r, "mvoteGranted |-> "); rt_s(r, m->a ? "TRUE" : "FALSE"); rt_s(r, ", mlog |-> "); rt_log(r, m->mlog);
        rt_s(r, ", ");
        break;
    case AEREQ:
        rt_s(r, "mprevLogIndex |-> "); rt_u(r, m->a); rt_s(r, ", mprevLogTerm |-> "); rt_u(r, m->b);
        rt_s(r, ", mentries |-> ");
        if (m->d) { rt_s(r, "<<[term |-> "); rt_u(r, m->et); rt_s(r, ", value |-> v"); rt_u(r, m->ev + 1u); rt_s(r, "]>>"); }
        else rt_s(r, "<<>>");
        rt_s(r, ", mlog |-> "); rt_log(r, m->mlog); rt_s(r, ", mcommitIndex |-> "); rt_u(r, m->c); rt_s(r, ", ");
        break;
    default:
        rt_s(r, "msuccess |-> "); rt_s(r, m->a ? "TRUE" : "FALSE"); rt_s(r, ", mmatchIndex |-> "); rt_u(r, m->b);
        rt_s(r, ", ");
    }
    rt_s(r, "msource |-> "); rt_srv(r, pi[m->src]); rt_s(r, ", mdest |-> "); rt_srv(r, pi[m->dst]); rt_s(r, "]");
    rt_s(r, " :> "); rt_u(r, (unsigned)cnt);
}
/* One election record of the image pi(s). */
static void rt_elec(RText *r, const Elec *e, const int *pi, int N) {
    rt_s(r, "[eterm |-> "); rt_u(r, e->term); rt_s(r, ", eleader |-> "); rt_srv(r, pi[e->leader]);
    rt_s(r, ", elog |-> "); rt_log(r, e->elog); rt_s(r, ", evotes |-> "); rt_srvset(r, perm_mask(e->votes, pi, N), N);
    rt_s(r, ", evoterLog |-> ");
    const int vlp = perm_mask(e->vlp, pi, N);
    if (!vlp) { rt_s(r, "<<>>"); }
    else {
        Log vl[NMAX];
        for (int j = 0; j < N; j++) vl[pi[j]] = e->vl[j];
        rt_s(r, "(");
        int first = 1;
        for (int q = 0; q < N; q++)
            if (vlp >> q & 1) { if (!first) rt_s(r, " @@ "); rt_srv(r, q); rt_s(r, " :> "); rt_log(r, vl[q]); first = 0; }
        rt_s(r, ")");
    }
    rt_s(r, "]");
}
typedef struct { const char *p; size_t n; } Item;
static int item_cmp(const void *a, const void *b) {
    const Item *x = (const Item *)a, *y = (const Item *)b;
    const int d = memcmp(x->p, y->p, x->n < y->n ? x->n : y->n);
    return d ? d : (x->n < y->n ? -1 : x->n > y->n);
}
/* "\n/\\ messages = ...\n/\\ elections = ..." of the image pi(s) into r
 * (items rendered into `scratch`, sorted by text); 1 if above best */
static int rt_bag(const orc_cfg *c, const State *s, const int *pi, RText *r, char *scratch) {
    const int N = c->n_server;
    Item it[KMAX > EMAX ? KMAX : EMAX];
    RText w = {scratch, 0, NULL, 0, -1};
    for (int k = 0; k < s->nmsg; k++) {
        const size_t b = w.n;
        rt_msg(&w, &s->msg[k], s->cnt[k], pi);
        it[k].p = scratch + b; it[k].n = w.n - b;
    }
    qsort(it, (size_t)s->nmsg, sizeof(Item), item_cmp);
    if (rt_s(r, "\n/\\ messages = ")) return 1;
    if (!s->nmsg) { if (rt_s(r, "<<>>")) return 1; }
    else {
        if (rt_s(r, "(")) return 1;
        for (int k = 0; k < s->nmsg; k++) if ((k && rt_s(r, " @@ ")) || rt_put(r, it[k].p, it[k].n)) return 1;
        if (rt_s(r, ")")) return 1;
    }
    w.n = 0;
    for (int k = 0; k < s->nelec; k++) {
        const size_t b = w.n;
        rt_elec(&w, &s->elec[k], pi, N);
        it[k].p = scratch + b; it[k].n = w.n - b;
    }
    qsort(it, (size_t)s->nelec, sizeof(Item), item_cmp);
    if (rt_s(r, "\n/\\ elections = ")) return 1;
    if (!s->nelec) return rt_s(r, "{}");
    if (rt_s(r, "{")) return 1;
    for (int k = 0; k < s->nelec; k++) if ((k && rt_s(r, ", ")) || rt_put(r, it[k].p, it[k].n)) return 1;
    return rt_s(r, "}");
}
static char *state_text(const orc_cfg *c, const State *s);
/* The orbit text of s (malloc'd).  The rotated text of an image pi(s) is
 * its ten per-server lines, then messages, elections (and allLogs, the same
 * for every image: left out of the comparison).  Exact shortcut: the first
 * two rotated lines (currentTerm, state) print one relabel-free token per
 * position -- a decimal term, a quoted role, neither with a token a proper
 * prefix of another that continues below the delimiters " @@ " / ")" -- so
 * their least text puts the servers in (term text, role text) order and
 * every image that does not is above it there; only the orderings of servers
 * tied on (term, role) are compared, from the third line on.  (The value
 * oracle, raft_values.orbit_text, compares all N! images in full.) */
static char *orbit_text(const orc_cfg *c, const State *s) {
    const int N = c->n_server;
    static const int RRANK[3] = {1, 0, 2};   /* "Candidate" < "Follower" < "Leader" */
    int key[NMAX], sg[NMAX], pi[NMAX], bpi[NMAX], gb[NMAX + 1];
    for (int i = 0; i < N; i++) {
        const int t = s->s[i].term;
        key[i] = ((t >= 10 ? t / 10 : t) * 11 + (t >= 10 ? t % 10 + 1 : 0)) * 4 + RRANK[s->s[i].role];
    }
    const int ng = sg_first(key, N, sg, gb);
    static __thread char *work;       /* two rotated texts + item scratch, per worker thread */
    const size_t cap = 1 << 18;
    if (!work) work = (char *)malloc(3 * cap);
    char *bufs[2] = {work, work + cap}, *scratch = work + 2 * cap;
    int bi = -1;
    size_t bn = 0;
    for (;;) {
        for (int p = 0; p < N; p++) pi[sg[p]] = p;
        const int ci = bi < 0 ? 0 : bi ^ 1;
        RText q = {bufs[ci], 0, bi < 0 ? NULL : bufs[bi], bn, bi < 0 ? -1 : 0};
        if (!rt_servers(c, s, pi, sg, &q, 2) && !rt_bag(c, s, pi, &q, scratch) && q.st < 0) {
            bi = ci; bn = q.n;
            memcpy(bpi, pi, sizeof pi);
        }
        if (!sg_next(sg, gb, ng)) break;
    }
    State *tmp = (State *)malloc(sizeof(State));
    permute_state(c, s, bpi, tmp);
    char *out = state_text(c, tmp);
    free(tmp);
    return out;
}

/* ------------------------------------------------------- text printing -- */
/* Canonical TLC-like value text; identical to oracle/raft_values.py::state_text. */
typedef struct { char *p; size_t n, cap; } Str;
static void sput(Str *s, const char *t) {
    size_t l = strlen(t);
    if (s->n + l + 1 > s->cap) {
        s->cap = (s->n + l + 1) * 2 + 256;
        s->p = (char *)realloc(s->p, s->cap);
    }
    memcpy(s->p + s->n, t, l + 1);
    s->n += l;
}
static void sprintf_(Str *s, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void sprintf_(Str *s, const char *fmt, ...) {
    char buf[512];
    va_list ap; va_start(ap, fmt); vsnprintf(buf, sizeof buf, fmt, ap); va_end(ap);
    sput(s, buf);
}
static void text_log(Str *s, Log l) {
    int n = log_len(l);
    if (!n) { sput(s, "<<>>"); return; }
    sput(s, "<<");
    for (int k = 1; k <= n; k++) {
        if (k > 1) sput(s, ", ");
        sprintf_(s, "[term |-> %d, value |-> v%d]", log_term(l, k), log_val(l, k) + 1);
    }
    sput(s, ">>");
}
static void text_srvset(Str *s, int mask, int N) {
    sput(s, "{");
    int first = 1;
    for (int j = 0; j < N; j++) if (mask >> j & 1) { if (!first) sput(s, ", "); sprintf_(s, "s%d", j + 1); first = 0; }
    sput(s, "}");
}
static void text_vl(Str *s, int vlp, const Log *vl, int N) {
    if (!vlp) { sput(s, "<<>>"); return; }
    sput(s, "(");
    int first = 1;
    for (int j = 0; j < N; j++) if (vlp >> j & 1) {
        if (!first) sput(s, " @@ ");
        sprintf_(s, "s%d :> ", j + 1); text_log(s, vl[j]); first = 0;
    }
    sput(s, ")");
}
static void text_msg(Str *s, const Msg *m) {
    static const char *TN[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest", "AppendEntriesResponse"};
    sprintf_(s, "[mtype |-> \"%s\", mterm |-> %d, ", TN[m->type], m->term);
    switch (m->type) {
    case RVREQ: sprintf_(s, "mlastLogTerm |-> %d, mlastLogIndex |-> %d, ", m->a, m->b); break;
    case RVRESP: sprintf_(s, "mvoteGranted |-> %s, mlog |-> ", m->a ? "TRUE" : "FALSE"); text_log(s, m->mlog); sput(s, ", "); break;
    case AEREQ:
        sprintf_(s, "mprevLogIndex |-> %d, mprevLogTerm |-> %d, mentries |-> ", m->a, m->b);
        if (m->d) sprintf_(s, "<<[term |-> %d, value |-> v%d]>>", m->et, m->ev + 1); else sput(s, "<<>>");
        sput(s, ", mlog |-> "); text_log(s, m->mlog);
        sprintf_(s, ", mcommitIndex |-> %d, ", m->c);
        break;
    case AERESP: sprintf_(s, "msuccess |-> %s, mmatchIndex |-> %d, ", m->a ? "TRUE" : "FALSE", m->b); break;
    }
    sprintf_(s, "msource |-> s%d, mdest |-> s%d]", m->src + 1, m->dst + 1);
}
static int cmpstr(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

/* Sort `n` strings and join as "{a, b}" or "(a :> c @@ ...)" */
static void text_sorted_join(Str *out, char **items, int n, const char *open, const char *sep, const char *close, const char *empty) {
    if (!n) { sput(out, empty); return; }
    qsort(items, (size_t)n, sizeof(char *), cmpstr);
    sput(out, open);
    for (int k = 0; k < n; k++) { if (k) sput(out, sep); sput(out, items[k]); }
    sput(out, close);
}

static char *state_text(const orc_cfg *c, const State *s) {
    const int N = c->n_server;
    Str o = {0};
    char **items = (char **)malloc(sizeof(char *) * (size_t)(s->nmsg + s->nelec + s->nall + 1));
    /* messages */
    for (int k = 0; k < s->nmsg; k++) {
        Str t = {0}; text_msg(&t, &s->msg[k]); sprintf_(&t, " :> %d", s->cnt[k]); items[k] = t.p;
    }
    sput(&o, "/\\ messages = ");
    text_sorted_join(&o, items, s->nmsg, "(", " @@ ", ")", "<<>>");
    for (int k = 0; k < s->nmsg; k++) free(items[k]);
    /* elections */
    for (int k = 0; k < s->nelec; k++) {
        const Elec *e = &s->elec[k];
        Str t = {0};
        sprintf_(&t, "[eterm |-> %d, eleader |-> s%d, elog |-> ", e->term, e->leader + 1);
        text_log(&t, e->elog); sput(&t, ", evotes |-> "); text_srvset(&t, e->votes, N);
        sput(&t, ", evoterLog |-> "); text_vl(&t, e->vlp, e->vl, N); sput(&t, "]");
        items[k] = t.p;
    }
    sput(&o, "\n/\\ elections = ");
    text_sorted_join(&o, items, s->nelec, "{", ", ", "}", "{}");
    for (int k = 0; k < s->nelec; k++) free(items[k]);
    /* allLogs */
    for (int k = 0; k < s->nall; k++) { Str t = {0}; text_log(&t, s->all[k]); items[k] = t.p; }
    sput(&o, "\n/\\ allLogs = ");
    text_sorted_join(&o, items, s->nall, "{", ", ", "}", "{}");
    for (int k = 0; k < s->nall; k++) free(items[k]);
    free(items);
    static const char *RN[3] = {"\"Follower\"", "\"Candidate\"", "\"Leader\""};
#define PERSRV(name, body)                                           \
    do {                                                             \
        sput(&o, "\n/\\ " name " = (");                              \
        for (int i = 0; i < N; i++) {                                \
            const Srv *v = &s->s[i]; (void)v;                        \
            if (i) sput(&o, " @@ ");                                 \
            sprintf_(&o, "s%d :> ", i + 1);                          \
            body;                                                    \
        }                                                            \
        sput(&o, ")");                                               \
    } while (0)
    PERSRV("currentTerm", sprintf_(&o, "%d", v->term));
    PERSRV("state", sput(&o, RN[v->role]));
    PERSRV("votedFor", if (v->voted == NIL) sput(&o, "\"Nil\""); else sprintf_(&o, "s%d", v->voted + 1));
    PERSRV("log", text_log(&o, v->log));
    PERSRV("commitIndex", sprintf_(&o, "%d", v->commit));
    PERSRV("votesResponded", text_srvset(&o, v->vresp, N));
    PERSRV("votesGranted", text_srvset(&o, v->vgrant, N));
    PERSRV("voterLog", text_vl(&o, v->vlp, v->vl, N));
    PERSRV("nextIndex", { sput(&o, "("); for (int j = 0; j < N; j++) { if (j) sput(&o, " @@ "); sprintf_(&o, "s%d :> %d", j + 1, v->next[j]); } sput(&o, ")"); });
    PERSRV("matchIndex", { sput(&o, "("); for (int j = 0; j < N; j++) { if (j) sput(&o, " @@ "); sprintf_(&o, "s%d :> %d", j + 1, v->match[j]); } sput(&o, ")"); });
#undef PERSRV
    return o.p;
}

uint64_t orc_text_hash(const char *t) {  /* FNV-1a 64 of the text */
    uint64_t h = 0xcbf29ce484222325ULL;
    for (; *t; t++) { h ^= (uint8_t)*t; h *= 0x100000001b3ULL; }
    return h;
}

/* ----------------------------------------------------------- seen set -- */
#define NSHARD 4096
typedef struct {
    atomic_flag lock;
    uint64_t cap, n;
    uint64_t *k;   /* 2 words per slot, k[2i+1] == 0 => empty */
} Shard;

typedef struct { Shard sh[NSHARD]; } SeenSet;

static SeenSet *seen_new(void) {
    SeenSet *s = (SeenSet *)calloc(1, sizeof(SeenSet));
    for (int i = 0; i < NSHARD; i++) {
        s->sh[i].cap = 64;
        s->sh[i].k = (uint64_t *)calloc(2 * 64, sizeof(uint64_t));
        atomic_flag_clear(&s->sh[i].lock);
    }
    return s;
}
static void seen_free(SeenSet *s) {
    for (int i = 0; i < NSHARD; i++) free(s->sh[i].k);
    free(s);
}
static int shard_put_nolock(Shard *sh, uint64_t h1, uint64_t h2) {
    uint64_t mask = sh->cap - 1;
    uint64_t i = (h1 >> 12) & mask;
    for (;;) {
        uint64_t *e = &sh->k[2 * i];
        if (e[1] == 0) { e[0] = h1; e[1] = h2; sh->n++; return 1; }
        if (e[0] == h1 && e[1] == h2) return 0;
        i = (i + 1) & mask;
    }
}
/* returns 1 if newly inserted */
static int seen_put(SeenSet *s, uint64_t h1, uint64_t h2) {
    Shard *sh = &s->sh[h1 & (NSHARD - 1)];
    while (atomic_flag_test_and_set_explicit(&sh->lock, memory_order_acquire)) {}
    if ((sh->n + 1) * 10 > sh->cap * 7) {
        uint64_t oc = sh->cap; uint64_t *ok = sh->k;
        sh->cap = oc * 2; sh->n = 0;
        sh->k = (uint64_t *)calloc(2 * sh->cap, sizeof(uint64_t));
        for (uint64_t i = 0; i < oc; i++) if (ok[2 * i + 1]) shard_put_nolock(sh, ok[2 * i], ok[2 * i + 1]);
        free(ok);
    }
    int r = shard_put_nolock(sh, h1, h2);
    atomic_flag_clear_explicit(&sh->lock, memory_order_release);
    return r;
}

/* -------------------------------------------------------- arena (level) -- */
typedef struct {
    uint8_t *buf; size_t n, cap;
    uint64_t *off; uint64_t *parent; uint32_t *act; size_t cnt, ccap;
} Arena;
static void arena_push(Arena *a, const uint8_t *p, size_t len, uint64_t parent, uint32_t act) {
    if (a->n + len > a->cap) { a->cap = (a->n + len) * 2 + 4096; a->buf = (uint8_t *)realloc(a->buf, a->cap); }
    if (a->cnt + 1 > a->ccap) {
        a->ccap = a->ccap * 2 + 1024;
        a->off = (uint64_t *)realloc(a->off, a->ccap * 8);
        a->parent = (uint64_t *)realloc(a->parent, a->ccap * 8);
        a->act = (uint32_t *)realloc(a->act, a->ccap * 4);
    }
    memcpy(a->buf + a->n, p, len);
    a->off[a->cnt] = a->n; a->parent[a->cnt] = parent; a->act[a->cnt] = act; a->cnt++;
    a->n += len;
}
static void arena_free(Arena *a) { free(a->buf); free(a->off); free(a->parent); free(a->act); memset(a, 0, sizeof *a); }

/* ---------------------------------------------------------------- BFS -- */
typedef struct {
    const orc_cfg *c;
    SeenSet *seen;
    const Arena *cur;
    atomic_size_t next_item;
    Arena *outs;       /* one per thread */
    uint64_t *gen;     /* per thread */
    uint64_t *cover;   /* per thread x A_COUNT: generated per action family */
    int nthreads;
    atomic_int viol;   /* violated invariant mask (first) */
    atomic_int stop;
    /* violation site */
    pthread_mutex_t vmu;
    uint64_t v_parent; int v_action, v_arg, v_inmodel; uint8_t *v_state; size_t v_len;
    uint64_t level_base;
    int check_text_hash;
    uint64_t *text_hash; /* per thread */
    int count_only;      /* the last level of a max_levels prefix: count new states, keep none */
    uint64_t *nnew;      /* per thread: new states of the level */
    uint64_t *max_bytes, *max_msgs;  /* per thread: largest new state (serialised bytes, bag slots) */
} Bfs;

typedef struct { Bfs *b; int tid; uint64_t parent_idx; uint8_t *ser; } EmitCtx;

static void bfs_emit(void *ud, const State *t, int action, int arg) {
    EmitCtx *e = (EmitCtx *)ud;
    Bfs *b = e->b;
    b->gen[e->tid]++;
    b->cover[e->tid * A_COUNT + action]++;
    int inm = in_model(b->c, t);
    int isnew = 0;
    size_t len = 0;
    if (inm) {
        uint64_t h1, h2;
        if (b->c->symmetry) {  /* orbit key for the seen set; the state itself is explored */
            len = serialize_canon(b->c, t, e->ser);
            hash128(e->ser, len, &h1, &h2);
        }
        len = serialize(b->c, t, e->ser);
        if (!b->c->symmetry) hash128(e->ser, len, &h1, &h2);
        isnew = seen_put(b->seen, h1, h2);
        if (isnew) {
            b->nnew[e->tid]++;
            if (!b->count_only)
                arena_push(&b->outs[e->tid], e->ser, len, e->parent_idx, (uint32_t)(action << 16 | arg));
            if (b->check_text_hash) {   /* SYMMETRY: the orbit text */
                char *tx = b->c->symmetry ? orbit_text(b->c, t) : state_text(b->c, t);
                b->text_hash[e->tid] += orc_text_hash(tx);
                free(tx);
            }
            /* (every new state, the count-only last level's included) */
            if (len > b->max_bytes[e->tid]) b->max_bytes[e->tid] = len;
            if ((uint64_t)t->nmsg > b->max_msgs[e->tid]) b->max_msgs[e->tid] = (uint64_t)t->nmsg;
        }
    }
    if (!inm || isnew) {
        int bad = check_inv(b->c, t);
        if (bad) {
            pthread_mutex_lock(&b->vmu);
            if (!atomic_load(&b->viol)) {
                atomic_store(&b->viol, bad);
                b->v_parent = e->parent_idx; b->v_action = action; b->v_arg = arg; b->v_inmodel = inm;
                if (!inm) len = serialize(b->c, t, e->ser);
                b->v_state = (uint8_t *)malloc(len); memcpy(b->v_state, e->ser, len); b->v_len = len;
            }
            pthread_mutex_unlock(&b->vmu);
        }
    }
}

static void *bfs_worker(void *arg) {
    EmitCtx ec;
    ec.b = ((EmitCtx *)arg)->b; ec.tid = ((EmitCtx *)arg)->tid;
    Bfs *b = ec.b;
    State *s = (State *)malloc(sizeof(State));
    State *t = (State *)malloc(sizeof(State));
    State *base = (State *)malloc(sizeof(State));
    ec.ser = (uint8_t *)malloc(1 << 20);
    const size_t CH = 64;
    for (;;) {
        size_t i0 = atomic_fetch_add(&b->next_item, CH);
        if (i0 >= b->cur->cnt) break;
        size_t i1 = i0 + CH < b->cur->cnt ? i0 + CH : b->cur->cnt;
        for (size_t i = i0; i < i1; i++) {
            deserialize(b->c, b->cur->buf + b->cur->off[i], s);
            ec.parent_idx = b->level_base + i;
            expand(b->c, s, base, t, bfs_emit, &ec);
        }
    }
    free(s); free(t); free(base); free(ec.ser);
    return NULL;
}

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int orc_bfs(const orc_cfg *c, int nthreads, int keep_trace, int text_hash, orc_result *r) {
    memset(r, 0, sizeof *r);
    if (c->n_server < 1 || c->n_server > NMAX || c->max_log + 1 > LCAP || c->max_term > 14 || c->n_value > 15)
        return ORC_E_CONFIG;
    if (nthreads < 1) nthreads = 1;
    g_overflow = 0; g_spec_error = 0;
    double t0 = now_s();
    Bfs b; memset(&b, 0, sizeof b);
    b.c = c; b.seen = seen_new(); b.nthreads = nthreads; b.check_text_hash = text_hash;
    pthread_mutex_init(&b.vmu, NULL);
    b.outs = (Arena *)calloc((size_t)nthreads, sizeof(Arena));
    b.gen = (uint64_t *)calloc((size_t)nthreads, 8);
    b.cover = (uint64_t *)calloc((size_t)nthreads * A_COUNT, 8);
    b.text_hash = (uint64_t *)calloc((size_t)nthreads, 8);
    b.nnew = (uint64_t *)calloc((size_t)nthreads, 8);
    b.max_bytes = (uint64_t *)calloc((size_t)nthreads, 8);
    b.max_msgs = (uint64_t *)calloc((size_t)nthreads, 8);

    /* all levels (kept only when tracing) */
    Arena *levels = (Arena *)calloc(ORC_MAX_LEVELS + 1, sizeof(Arena));
    uint64_t *level_base = (uint64_t *)calloc(ORC_MAX_LEVELS + 1, 8);
    State *s0 = (State *)malloc(sizeof(State));
    uint8_t *ser = (uint8_t *)malloc(1 << 20);
    init_state(c, s0);
    size_t len = serialize_canon(c, s0, ser);
    uint64_t h1, h2; hash128(ser, len, &h1, &h2);
    seen_put(b.seen, h1, h2);
    len = serialize(c, s0, ser);
    arena_push(&levels[0], ser, len, UINT64_MAX, 0);
    r->n_levels = 1;
    r->level_new[0] = 1; r->level_gen[0] = 1;
    if (text_hash) {
        char *tx = c->symmetry ? orbit_text(c, s0) : state_text(c, s0);
        r->level_text_hash[0] = orc_text_hash(tx);
        free(tx);
    }
    r->max_state_bytes = len;
    r->distinct = 1; r->generated = 1;
    int bad0 = check_inv(c, s0);
    int cur = 0;
    int rc = ORC_OK;
    if (bad0) { r->violated = bad0; rc = ORC_VIOLATION; }
    while (rc == ORC_OK) {
        b.cur = &levels[cur];
        b.level_base = level_base[cur];
        atomic_store(&b.next_item, 0);
        memset(b.gen, 0, 8 * (size_t)nthreads);
        memset(b.text_hash, 0, 8 * (size_t)nthreads);
        memset(b.nnew, 0, 8 * (size_t)nthreads);
        b.count_only = c->max_levels > 0 && r->n_levels + 1 >= c->max_levels && !keep_trace;
        pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
        EmitCtx *ecs = (EmitCtx *)calloc((size_t)nthreads, sizeof(EmitCtx));
        for (int k = 0; k < nthreads; k++) { ecs[k].b = &b; ecs[k].tid = k; pthread_create(&th[k], NULL, bfs_worker, &ecs[k]); }
        for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
        free(th); free(ecs);
        uint64_t gen = 0, nnew = 0, th_sum = 0;
        for (int k = 0; k < nthreads; k++) { gen += b.gen[k]; nnew += b.nnew[k]; th_sum += b.text_hash[k]; }
        r->generated += gen;
        r->distinct += nnew;
        if (g_overflow) { rc = ORC_E_OVERFLOW; break; }
        if (g_spec_error) { rc = ORC_E_SPEC; break; }
        if (r->n_levels >= ORC_MAX_LEVELS) { rc = ORC_E_OVERFLOW; break; }
        int L = r->n_levels;
        r->level_new[L] = nnew; r->level_gen[L] = gen; r->level_text_hash[L] = th_sum;
        r->n_levels++;
        /* merge thread arenas into the next level */
        Arena *nx = &levels[cur + 1];
        level_base[cur + 1] = level_base[cur] + levels[cur].cnt;
        for (int k = 0; k < nthreads; k++) {
            Arena *a = &b.outs[k];
            for (size_t q = 0; q < a->cnt; q++) {
                size_t l2 = (q + 1 < a->cnt ? a->off[q + 1] : a->n) - a->off[q];
                arena_push(nx, a->buf + a->off[q], l2, a->parent[q], a->act[q]);
            }
            arena_free(a);
        }
        for (int k = 0; k < nthreads; k++) {   /* (tracked per new state: the count-only level too) */
            if (b.max_bytes[k] > r->max_state_bytes) r->max_state_bytes = b.max_bytes[k];
            if (b.max_msgs[k] > r->max_msgs) r->max_msgs = b.max_msgs[k];
        }
        if (atomic_load(&b.viol)) { r->violated = atomic_load(&b.viol); rc = ORC_VIOLATION; }
        if (!keep_trace) { arena_free(&levels[cur]); }
        cur++;
        if (c->verbose) {
            fprintf(stderr, "level %d: new %llu generated %llu distinct %llu (%.1fs)\n", L + 1,
                    (unsigned long long)nnew, (unsigned long long)gen, (unsigned long long)r->distinct, now_s() - t0);
        }
        if (nnew == 0) break;
        if (c->max_distinct && r->distinct > c->max_distinct) { rc = ORC_E_BUDGET; break; }
        if (c->max_levels && r->n_levels >= c->max_levels) { rc = ORC_E_BUDGET; break; }
    }
    r->depth = 0;
    for (int L = 0; L < r->n_levels; L++) if (r->level_new[L]) r->depth = L + 1;
    for (int k = 0; k < nthreads; k++)
        for (int a = 0; a < A_COUNT && a < ORC_MAX_ACTIONS; a++) r->coverage[a] += b.cover[k * A_COUNT + a];
    /* counterexample trace (texts), init -> bad */
    if (rc == ORC_VIOLATION && keep_trace) {
        Str tr = {0};
        State *st = (State *)malloc(sizeof(State));
        /* collect chain of global indices */
        uint64_t chain[ORC_MAX_LEVELS + 2]; int nc = 0;
        uint64_t gi = bad0 ? 0 : b.v_parent;
        for (;;) {
            chain[nc++] = gi;
            int L = 0;
            while (L + 1 <= cur && level_base[L + 1] <= gi && levels[L + 1].cnt) L++;
            uint64_t p = levels[L].parent[gi - level_base[L]];
            if (p == UINT64_MAX) break;
            gi = p;
        }
        for (int q = nc - 1; q >= 0; q--) {
            int L = 0;
            while (L + 1 <= cur && level_base[L + 1] <= chain[q] && levels[L + 1].cnt) L++;
            uint64_t li = chain[q] - level_base[L];
            deserialize(c, levels[L].buf + levels[L].off[li], st);
            char *tx = state_text(c, st);
            uint32_t act = levels[L].act[li];
            if (L == 0) sput(&tr, "<Initial predicate>\n");
            else sprintf_(&tr, "<%s>\n", ACTION_NAME[act >> 16]);
            sput(&tr, tx); sput(&tr, "\n\n");
            free(tx);
        }
        if (!bad0) {
            deserialize(c, b.v_state, st);
            char *tx = state_text(c, st);
            sprintf_(&tr, "<%s>\n", ACTION_NAME[b.v_action]);
            sput(&tr, tx); sput(&tr, "\n\n");
            free(tx);
        }
        r->trace_len = nc + (bad0 ? 0 : 1);
        r->trace_text = tr.p;
        free(st);
    }
    for (int L = 0; L <= cur && L <= ORC_MAX_LEVELS; L++) arena_free(&levels[L]);
    free(levels); free(level_base);
    for (int k = 0; k < nthreads; k++) arena_free(&b.outs[k]);
    free(b.outs); free(b.gen); free(b.cover); free(b.text_hash); free(b.nnew); free(b.max_bytes); free(b.max_msgs);
    free(b.v_state);
    seen_free(b.seen);
    free(s0); free(ser);
    r->seconds = now_s() - t0;
    return rc;
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------- lockstep random walk -- */
/* A walk handle holds one current state; the test harness lists the texts of
 * its successors and moves to the successor with a given text. */
typedef struct {
    orc_cfg c;
    State cur;
    State tmp, base;
    Str texts;     /* successor texts, '\x1e'-separated */
    int nsucc;
    State *succ;   /* successors */
    int cap;
    int *inmodel;
} Walk;

static void walk_emit(void *ud, const State *t, int action, int arg) {
    (void)action; (void)arg;
    Walk *w = (Walk *)ud;
    if (w->nsucc >= w->cap) {
        w->cap = w->cap * 2 + 64;
        w->succ = (State *)realloc(w->succ, sizeof(State) * (size_t)w->cap);
        w->inmodel = (int *)realloc(w->inmodel, sizeof(int) * (size_t)w->cap);
    }
    state_copy(&w->succ[w->nsucc], t);
    w->inmodel[w->nsucc] = in_model(&w->c, t);
    w->nsucc++;
}

void *orc_walk_new(const orc_cfg *c) {
    Walk *w = (Walk *)calloc(1, sizeof(Walk));
    w->c = *c;
    init_state(c, &w->cur);
    return w;
}
void orc_walk_free(void *h) {
    Walk *w = (Walk *)h;
    free(w->succ); free(w->inmodel); free(w->texts.p); free(w);
}
/* Writes "in_model\x1ftext\x1e" per successor. Returns #successors or -needed bytes. */
long orc_walk_successors(void *h, char *buf, size_t cap) {
    Walk *w = (Walk *)h;
    w->nsucc = 0;
    g_overflow = 0; g_spec_error = 0;
    expand(&w->c, &w->cur, &w->base, &w->tmp, walk_emit, w);
    if (g_overflow) return ORC_E_OVERFLOW;
    if (g_spec_error) return ORC_E_SPEC;
    w->texts.n = 0;
    sput(&w->texts, "");
    for (int k = 0; k < w->nsucc; k++) {
        char *tx = state_text(&w->c, &w->succ[k]);
        sput(&w->texts, w->inmodel[k] ? "1\x1f" : "0\x1f");
        sput(&w->texts, tx); sput(&w->texts, "\x1e");
        free(tx);
    }
    if (w->texts.n + 1 > cap) return -(long)(w->texts.n + 1);
    memcpy(buf, w->texts.p, w->texts.n + 1);
    return w->nsucc;
}
/* Move to the successor whose text equals `text`. Returns 0 or -1. */
int orc_walk_goto(void *h, const char *text) {
    Walk *w = (Walk *)h;
    for (int k = 0; k < w->nsucc; k++) {
        char *tx = state_text(&w->c, &w->succ[k]);
        int eq = strcmp(tx, text) == 0;
        free(tx);
        if (eq) { state_copy(&w->cur, &w->succ[k]); return 0; }
    }
    return -1;
}
long orc_walk_text(void *h, char *buf, size_t cap) {
    Walk *w = (Walk *)h;
    char *tx = state_text(&w->c, &w->cur);
    size_t l = strlen(tx);
    if (l + 1 > cap) { free(tx); return -(long)(l + 1); }
    memcpy(buf, tx, l + 1);
    free(tx);
    return (long)l;
}
int orc_walk_inv(void *h) { Walk *w = (Walk *)h; return check_inv(&w->c, &w->cur); }

/* SYMMETRY lockstep walks: the orbit text (see orbit_text) of each successor
 * listed by the last orc_walk_successors, '\x1e'-separated, and the hex
 * 128-bit hash of its least orbit serialisation (the oracle's seen-set key),
 * as "hash\x1ftext\x1e".  Returns #successors or -needed bytes. */
long orc_walk_orbits(void *h, char *buf, size_t cap) {
    Walk *w = (Walk *)h;
    Str o = {0};
    sput(&o, "");
    uint8_t *ser = (uint8_t *)malloc(1 << 17);
    for (int k = 0; k < w->nsucc; k++) {
        size_t len = serialize_canon(&w->c, &w->succ[k], ser);
        uint64_t h1, h2;
        hash128(ser, len, &h1, &h2);
        sprintf_(&o, "%016llx%016llx\x1f", (unsigned long long)h1, (unsigned long long)h2);
        char *tx = orbit_text(&w->c, &w->succ[k]);
        sput(&o, tx); sput(&o, "\x1e");
        free(tx);
    }
    free(ser);
    long r = (long)w->nsucc;
    if (o.n + 1 > cap) r = -(long)(o.n + 1);
    else memcpy(buf, o.p, o.n + 1);
    free(o.p);
    return r;
}

/* ------------------------------------------- text parser + dedup (CPU leg) -- */
/* The CPU baseline of the synthetic microbench (BASELINE configs[4]):
 * arbitrary states given as TLC value text (the product's random rows, printed
 * by rtla_random_texts) are parsed into this oracle's own representation and
 * run through Next + dedup: generated successors, probes (in-model successors
 * that differ from their parent) and distinct new successors, with the seen
 * set kept across batches -- the counts the GPU's dedup kernel reports. */
typedef struct { const char *p; int err; } Rd;
static void rd_ex(Rd *q, const char *lit) {
    const size_t n = strlen(lit);
    if (strncmp(q->p, lit, n)) q->err = 1; else q->p += n;
}
static int rd_at(Rd *q, const char *lit) { return !strncmp(q->p, lit, strlen(lit)); }
static int rd_int(Rd *q) {
    if (*q->p < '0' || *q->p > '9') { q->err = 1; return 0; }
    int v = 0;
    while (*q->p >= '0' && *q->p <= '9') v = v * 10 + (*q->p++ - '0');
    return v;
}
static int rd_srv(Rd *q) { rd_ex(q, "s"); return rd_int(q) - 1; }
static int rd_bool(Rd *q) {
    if (rd_at(q, "TRUE")) { q->p += 4; return 1; }
    rd_ex(q, "FALSE");
    return 0;
}
static Log rd_log(Rd *q) {
    if (rd_at(q, "<<>>")) { q->p += 4; return 0; }
    rd_ex(q, "<<");
    Log l = 0;
    for (int k = 0; !q->err && k < LCAP; k++) {
        rd_ex(q, "[term |-> "); const int t = rd_int(q);
        rd_ex(q, ", value |-> v"); const int v = rd_int(q) - 1;
        rd_ex(q, "]");
        l = log_append(l, t, v);
        if (!rd_at(q, ", ")) break;
        q->p += 2;
    }
    rd_ex(q, ">>");
    return l;
}
static int rd_set(Rd *q) {
    rd_ex(q, "{");
    int m = 0;
    if (!rd_at(q, "}"))
        for (int k = 0; !q->err && k < NMAX; k++) {
            m |= 1 << rd_srv(q);
            if (!rd_at(q, ", ")) break;
            q->p += 2;
        }
    rd_ex(q, "}");
    return m;
}
static int rd_vl(Rd *q, Log *vl) {
    if (rd_at(q, "<<>>")) { q->p += 4; return 0; }
    rd_ex(q, "(");
    int m = 0;
    for (int k = 0; !q->err && k < NMAX; k++) {
        const int j = rd_srv(q);
        rd_ex(q, " :> ");
        if (j < 0 || j >= NMAX) { q->err = 1; break; }
        vl[j] = rd_log(q);
        m |= 1 << j;
        if (!rd_at(q, " @@ ")) break;
        q->p += 4;
    }
    rd_ex(q, ")");
    return m;
}
static void rd_msg(Rd *q, Msg *m, int *cnt) {
    static const char *TN[4] = {"RequestVoteRequest\"", "RequestVoteResponse\"", "AppendEntriesRequest\"",
                                "AppendEntriesResponse\""};
    memset(m, 0, sizeof *m);
    rd_ex(q, "[mtype |-> \"");
    int t = 0;
    while (t < 4 && !rd_at(q, TN[t])) t++;
    if (t == 4) { q->err = 1; return; }
    q->p += strlen(TN[t]);
    m->type = (uint8_t)t;
    rd_ex(q, ", mterm |-> "); m->term = (uint8_t)rd_int(q); rd_ex(q, ", ");
    switch (t) {
    case RVREQ:
        rd_ex(q, "mlastLogTerm |-> "); m->a = (uint8_t)rd_int(q);
        rd_ex(q, ", mlastLogIndex |-> "); m->b = (uint8_t)rd_int(q);
        break;
    case RVRESP:
        rd_ex(q, "mvoteGranted |-> "); m->a = (uint8_t)rd_bool(q);
        rd_ex(q, ", mlog |-> "); m->mlog = rd_log(q);
        break;
    case AEREQ:
        rd_ex(q, "mprevLogIndex |-> "); m->a = (uint8_t)rd_int(q);
        rd_ex(q, ", mprevLogTerm |-> "); m->b = (uint8_t)rd_int(q);
        rd_ex(q, ", mentries |-> ");
        if (rd_at(q, "<<>>")) { q->p += 4; }
        else {
            rd_ex(q, "<<[term |-> "); m->et = (uint8_t)rd_int(q);
            rd_ex(q, ", value |-> v"); m->ev = (uint8_t)(rd_int(q) - 1);
            rd_ex(q, "]>>"); m->d = 1;
        }
        rd_ex(q, ", mlog |-> "); m->mlog = rd_log(q);
        rd_ex(q, ", mcommitIndex |-> "); m->c = (uint8_t)rd_int(q);
        break;
    default:
        rd_ex(q, "msuccess |-> "); m->a = (uint8_t)rd_bool(q);
        rd_ex(q, ", mmatchIndex |-> "); m->b = (uint8_t)rd_int(q);
    }
    rd_ex(q, ", msource |-> "); m->src = (uint8_t)rd_srv(q);
    rd_ex(q, ", mdest |-> "); m->dst = (uint8_t)rd_srv(q);
    rd_ex(q, "] :> "); *cnt = rd_int(q);
}
/* Parse one state text (state_text's format) into s; 0 on success. */
static int parse_state(const orc_cfg *c, const char *text, State *s) {
    const int N = c->n_server;
    Rd q = {text, 0};
    memset(s, 0, sizeof *s);
    rd_ex(&q, "/\\ messages = ");
    if (rd_at(&q, "<<>>")) q.p += 4;
    else {
        rd_ex(&q, "(");
        while (!q.err) {
            Msg m; int cnt = 0, pos;
            rd_msg(&q, &m, &cnt);
            if (q.err || m.src >= N || m.dst >= N || cnt < 1 || s->nmsg >= KMAX || bag_find(s, &m, &pos)) return -1;
            memmove(&s->msg[pos + 1], &s->msg[pos], sizeof(Msg) * (s->nmsg - pos));
            memmove(&s->cnt[pos + 1], &s->cnt[pos], s->nmsg - pos);
            s->msg[pos] = m; s->cnt[pos] = (uint8_t)cnt; s->nmsg++;
            if (!rd_at(&q, " @@ ")) break;
            q.p += 4;
        }
        rd_ex(&q, ")");
    }
    rd_ex(&q, "\n/\\ elections = {");
    if (!rd_at(&q, "}"))
        while (!q.err) {
            Elec e; memset(&e, 0, sizeof e);
            rd_ex(&q, "[eterm |-> "); e.term = (uint8_t)rd_int(&q);
            rd_ex(&q, ", eleader |-> "); e.leader = (uint8_t)rd_srv(&q);
            rd_ex(&q, ", elog |-> "); e.elog = rd_log(&q);
            rd_ex(&q, ", evotes |-> "); e.votes = (uint8_t)rd_set(&q);
            rd_ex(&q, ", evoterLog |-> "); e.vlp = (uint8_t)rd_vl(&q, e.vl);
            rd_ex(&q, "]");
            if (q.err || s->nelec >= EMAX) return -1;
            elec_add(s, &e);
            if (!rd_at(&q, ", ")) break;
            q.p += 2;
        }
    rd_ex(&q, "}\n/\\ allLogs = {");
    if (!rd_at(&q, "}"))
        while (!q.err) {
            all_add(s, rd_log(&q));
            if (!rd_at(&q, ", ")) break;
            q.p += 2;
        }
    rd_ex(&q, "}");
    static const char *NAME[10] = {"currentTerm", "state", "votedFor", "log", "commitIndex", "votesResponded",
                                   "votesGranted", "voterLog", "nextIndex", "matchIndex"};
    for (int k = 0; k < 10 && !q.err; k++) {
        rd_ex(&q, "\n/\\ "); rd_ex(&q, NAME[k]); rd_ex(&q, " = (");
        for (int i = 0; i < N && !q.err; i++) {
            Srv *v = &s->s[i];
            if (i) rd_ex(&q, " @@ ");
            if (rd_srv(&q) != i) return -1;
            rd_ex(&q, " :> ");
            switch (k) {
            case 0: v->term = (uint8_t)rd_int(&q); break;
            case 1:
                if (rd_at(&q, "\"Follower\"")) { v->role = FOLLOWER; q.p += 10; }
                else if (rd_at(&q, "\"Candidate\"")) { v->role = CANDIDATE; q.p += 11; }
                else { rd_ex(&q, "\"Leader\""); v->role = LEADER; }
                break;
            case 2:
                if (rd_at(&q, "\"Nil\"")) { v->voted = NIL; q.p += 5; }
                else v->voted = (uint8_t)rd_srv(&q);
                break;
            case 3: v->log = rd_log(&q); break;
            case 4: v->commit = (uint8_t)rd_int(&q); break;
            case 5: v->vresp = (uint8_t)rd_set(&q); break;
            case 6: v->vgrant = (uint8_t)rd_set(&q); break;
            case 7: v->vlp = (uint8_t)rd_vl(&q, v->vl); break;
            default:
                rd_ex(&q, "(");
                for (int j = 0; j < N && !q.err; j++) {
                    if (j) rd_ex(&q, " @@ ");
                    if (rd_srv(&q) != j) return -1;
                    rd_ex(&q, " :> ");
                    if (k == 8) v->next[j] = (uint8_t)rd_int(&q); else v->match[j] = (uint8_t)rd_int(&q);
                }
                rd_ex(&q, ")");
            }
        }
        rd_ex(&q, ")");
    }
    return q.err || *q.p ? -1 : 0;
}

typedef struct {
    orc_cfg c;
    SeenSet *seen;
    uint64_t gen, probes, nnew;
} Dedup;
typedef struct {
    Dedup *d;
    const char *const *texts;
    size_t n;
    atomic_size_t next;
    atomic_int err;
    uint64_t *cnt;   /* per thread: gen, probes, new */
    int tid_next;
    pthread_mutex_t mu;
    State *states;   /* the inputs, parsed before the timed phase */
    int parse;       /* 1: the workers parse texts -> states; 0: they expand + deduplicate states */
} DedupJob;
typedef struct { DedupJob *j; int tid; uint8_t *pser; size_t plen; uint8_t *ser; } DedupEmit;
static void dedup_emit(void *ud, const State *t, int action, int arg) {
    (void)action; (void)arg;
    DedupEmit *e = (DedupEmit *)ud;
    uint64_t *cnt = e->j->cnt + 3 * e->tid;
    cnt[0]++;
    if (!in_model(&e->j->d->c, t)) return;
    const size_t len = serialize(&e->j->d->c, t, e->ser);
    if (len == e->plen && !memcmp(e->ser, e->pser, len)) return;   /* the parent itself */
    cnt[1]++;
    uint64_t h1, h2;
    hash128(e->ser, len, &h1, &h2);
    cnt[2] += (uint64_t)seen_put(e->j->d->seen, h1, h2);
}
static void *dedup_worker(void *arg) {
    DedupJob *j = (DedupJob *)arg;
    pthread_mutex_lock(&j->mu);
    DedupEmit e = {j, j->tid_next++, NULL, 0, NULL};
    pthread_mutex_unlock(&j->mu);
    State *t = (State *)malloc(sizeof(State)), *base = (State *)malloc(sizeof(State));
    e.pser = (uint8_t *)malloc(1 << 17);
    e.ser = (uint8_t *)malloc(1 << 17);
    for (;;) {
        const size_t i = atomic_fetch_add(&j->next, 1);
        if (i >= j->n) break;
        State *s = &j->states[i];
        if (j->parse) {
            if (parse_state(&j->d->c, j->texts[i], s)) { atomic_store(&j->err, 1); break; }
            continue;
        }
        e.plen = serialize(&j->d->c, s, e.pser);
        expand(&j->d->c, s, base, t, dedup_emit, &e);
    }
    free(t); free(base); free(e.pser); free(e.ser);
    return NULL;
}
void *orc_dedup_new(const orc_cfg *c) {
    Dedup *d = (Dedup *)calloc(1, sizeof(Dedup));
    d->c = *c;
    d->seen = seen_new();
    return d;
}
void orc_dedup_free(void *h) {
    Dedup *d = (Dedup *)h;
    if (!d) return;
    seen_free(d->seen);
    free(d);
}
/* Expand + dedup the states of `texts` ('\x1e'-terminated state texts, n of
 * them), threads workers; out[0..2] += generated, probes, new; *seconds =
 * the expand + dedup phase (the texts are parsed before it, untimed).
 * Returns 0, or -1 on a text it cannot parse. */
int orc_dedup_texts(void *h, const char *texts, size_t n, int threads, uint64_t *out, double *seconds) {
    Dedup *d = (Dedup *)h;
    g_overflow = 0; g_spec_error = 0;
    const char **v = (const char **)malloc(sizeof(char *) * (n ? n : 1));
    char *buf = strdup(texts);
    char *p = buf;
    for (size_t i = 0; i < n; i++) {
        v[i] = p;
        char *e = strchr(p, '\x1e');
        if (!e) { free(v); free(buf); return -1; }
        *e = 0;
        p = e + 1;
    }
    if (threads < 1) threads = 1;
    DedupJob j;
    memset(&j, 0, sizeof j);
    j.d = d; j.texts = v; j.n = n;
    atomic_store(&j.next, 0); atomic_store(&j.err, 0);
    j.cnt = (uint64_t *)calloc((size_t)threads * 3, 8);
    j.states = (State *)malloc(sizeof(State) * (n ? n : 1));
    pthread_mutex_init(&j.mu, NULL);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    /* the texts are parsed first, outside the timed phase (the GPU leg is
       handed packed rows: it parses nothing) */
    j.parse = 1;
    for (int k = 0; k < threads; k++) pthread_create(&th[k], NULL, dedup_worker, &j);
    for (int k = 0; k < threads; k++) pthread_join(th[k], NULL);
    j.parse = 0;
    j.tid_next = 0;
    atomic_store(&j.next, 0);
    const double t0 = now_s();
    if (!atomic_load(&j.err)) {
        for (int k = 0; k < threads; k++) pthread_create(&th[k], NULL, dedup_worker, &j);
        for (int k = 0; k < threads; k++) pthread_join(th[k], NULL);
    }
    if (seconds) *seconds = now_s() - t0;
    for (int k = 0; k < threads; k++)
        for (int x = 0; x < 3; x++) out[x] += j.cnt[3 * k + x];
    free(th); free(j.cnt); free(j.states); free(v); free(buf);
    pthread_mutex_destroy(&j.mu);
    return atomic_load(&j.err) || g_overflow || g_spec_error ? -1 : 0;
}
