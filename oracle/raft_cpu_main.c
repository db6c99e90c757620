/* raft_cpu_main.c -- CLI for the CPU oracle (TEST INFRASTRUCTURE ONLY). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "raft_cpu.h"

int main(int argc, char **argv) {
    orc_cfg c = {3, 1, 2, 1, 1, 0, 1, 0, 0, 0, 0};
    int threads = 8, trace = 0;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : "0";
        if (!strcmp(a, "-n")) { c.n_server = atoi(v); i++; }
        else if (!strcmp(a, "-v")) { c.n_value = atoi(v); i++; }
        else if (!strcmp(a, "-t")) { c.max_term = atoi(v); i++; }
        else if (!strcmp(a, "-l")) { c.max_log = atoi(v); i++; }
        else if (!strcmp(a, "-c")) { c.max_copies = atoi(v); i++; }
        else if (!strcmp(a, "-M")) { c.max_msgs = atoi(v); i++; }
        else if (!strcmp(a, "-i")) { c.inv_mask = atoi(v); i++; }
        else if (!strcmp(a, "-w")) { threads = atoi(v); i++; }
        else if (!strcmp(a, "-m")) { c.max_distinct = strtoull(v, 0, 10); i++; }
        else if (!strcmp(a, "-s")) { c.symmetry = 1; }
        else if (!strcmp(a, "-L")) { c.max_levels = atoi(v); i++; }
        else if (!strcmp(a, "--trace")) trace = 1;
        else if (!strcmp(a, "-q")) c.verbose = 0;
        else { fprintf(stderr, "unknown arg %s\n", a); return 2; }
    }
    orc_result *r = calloc(1, sizeof(orc_result));
    int rc = orc_bfs(&c, threads, trace, 0, r);
    printf("{\"rc\": %d, \"distinct\": %llu, \"generated\": %llu, \"depth\": %d, \"violated\": %d, "
           "\"max_msgs\": %llu, \"max_state_bytes\": %llu, \"seconds\": %.3f, \"threads\": %d, \"levels\": [",
           rc, (unsigned long long)r->distinct, (unsigned long long)r->generated, r->depth, r->violated,
           (unsigned long long)r->max_msgs, (unsigned long long)r->max_state_bytes, r->seconds, threads);
    for (int L = 0; L < r->n_levels; L++)
        printf("%s[%llu, %llu]", L ? ", " : "", (unsigned long long)r->level_new[L], (unsigned long long)r->level_gen[L]);
    printf("]}\n");
    if (r->trace_text) { fputs(r->trace_text, stderr); orc_free(r->trace_text); }
    free(r);
    return rc < 0 ? 1 : 0;
}
