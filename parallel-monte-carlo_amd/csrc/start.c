/*
 * start.c -- the `start` driver (reference: start.cu:169-272 main; energy trace as in
 * CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:566-709), written against the C ABI (pmc.h).
 *
 *   start [--cps 4] [--atoms 64] [--passes 1000] [--nmax 16] [--moves 10] [--beta 0.3]
 *         [--sigma 0.5] [--w 2.5] [--seed 1234] [--every 1] [--graph]
 *         [--dump FILE] [--save FILE] [--restart FILE]
 *
 * --dump writes create_dump frames (kernel.cu:510-536; the reference's VISUALISATION path) of the
 * initial state and after every --every sweeps; --save writes a PMCSNAP1 snapshot at the end;
 * --restart continues from a snapshot (its sweep index, state and statistics) instead of the
 * lattice, for --passes further sweeps.
 *
 * Prints "step: energy" lines like kernel.cu:643,695 (energy from the cell-list sum every
 * --every sweeps) and a final summary with acceptance ratio and trial-moves/s.  Compile-time
 * #defines of the reference (start.cu:14-24) become runtime flags.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pmc.h"

static void die(const char* what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, pmc_last_error());
    exit(1);
}

int main(int argc, char** argv) {
    pmc_params p;
    memset(&p, 0, sizeof(p));
    p.cps_x = 4; p.nmax = 16; p.n_moves = 10;
    p.w = 2.5f; p.beta = 0.3f; p.sigma = 0.5f; p.seed = 1234;
    long long atoms = 64;
    int passes = 1000, every = 1, graph = 0;
    const char *dump = NULL, *save = NULL, *restart = NULL;
    for (int i = 1; i < argc; ++i) {
        const char* a = argv[i];
        const char* v = (i + 1 < argc) ? argv[i + 1] : "0";
        if (!strcmp(a, "--cps")) { p.cps_x = atoi(v); ++i; }
        else if (!strcmp(a, "--atoms")) { atoms = atoll(v); ++i; }
        else if (!strcmp(a, "--passes")) { passes = atoi(v); ++i; }
        else if (!strcmp(a, "--nmax")) { p.nmax = atoi(v); ++i; }
        else if (!strcmp(a, "--moves")) { p.n_moves = atoi(v); ++i; }
        else if (!strcmp(a, "--beta")) { p.beta = (float)atof(v); ++i; }
        else if (!strcmp(a, "--sigma")) { p.sigma = (float)atof(v); ++i; }
        else if (!strcmp(a, "--w")) { p.w = (float)atof(v); ++i; }
        else if (!strcmp(a, "--seed")) { p.seed = strtoull(v, NULL, 10); ++i; }
        else if (!strcmp(a, "--every")) { every = atoi(v); ++i; }
        else if (!strcmp(a, "--graph")) { graph = 1; }
        else if (!strcmp(a, "--dump")) { dump = v; ++i; }
        else if (!strcmp(a, "--save")) { save = v; ++i; }
        else if (!strcmp(a, "--restart")) { restart = v; ++i; }
        else { fprintf(stderr, "unknown flag %s\n", a); return 2; }
    }
    if (every < 1) every = 1;

    pmc_ctx* ctx = NULL;
    int rc = pmc_create(&p, &ctx);
    if (rc) die("pmc_create", rc);
    uint32_t first = 0;
    if (restart) {
        if ((rc = pmc_load_snapshot(ctx, restart, &first))) die("pmc_load_snapshot", rc);
    } else if ((rc = pmc_init_lattice(ctx, atoms))) {
        die("pmc_init_lattice", rc);
    }
    if (dump && (rc = pmc_dump_frame(ctx, dump, 0, (int64_t)first))) die("pmc_dump_frame", rc);

    double e = 0.0;
    rc = pmc_energy(ctx, &e);
    if (rc) die("pmc_energy", rc);
    printf("0: %f\n", e);
    pmc_stats total;
    memset(&total, 0, sizeof(total));
    double seconds = 0.0;
    for (int s0 = 0; s0 < passes; s0 += every) {
        int k = (passes - s0) < every ? (passes - s0) : every;
        const int s = (int)first + s0;
        pmc_result r;
        if (graph) {
            pmc_stats a, b;
            if ((rc = pmc_stats_read(ctx, &a, 0))) die("pmc_stats_read", rc);
            if ((rc = pmc_run_graph(ctx, (uint32_t)s, k))) die("pmc_run_graph", rc);
            if ((rc = pmc_synchronize(ctx))) die("pmc_synchronize", rc);
            if ((rc = pmc_stats_read(ctx, &b, 0))) die("pmc_stats_read", rc);
            if ((rc = pmc_energy(ctx, &e))) die("pmc_energy", rc);
            total.accepted += b.accepted - a.accepted;
            total.trials += b.trials - a.trials;
            total.evaluated += b.evaluated - a.evaluated;
            total.de_fixed += b.de_fixed - a.de_fixed;
        } else {
            /* energies once per interval (for the trace line), not around every pmc_start */
            if ((rc = pmc_start_ex(ctx, (uint32_t)s, k, PMC_START_NO_ENERGY, &r))) die("pmc_start_ex", rc);
            if ((rc = pmc_energy(ctx, &e))) die("pmc_energy", rc);
            seconds += r.seconds;
            total.accepted += r.stats.accepted;
            total.trials += r.stats.trials;
            total.evaluated += r.stats.evaluated;
            total.de_fixed += r.stats.de_fixed;
        }
        printf("%d: %f\n", s + k, e);
        if (dump && (rc = pmc_dump_frame(ctx, dump, 1, (int64_t)(s + k)))) die("pmc_dump_frame", rc);
    }
    if (save && (rc = pmc_save_snapshot(ctx, save, first + (uint32_t)passes))) die("pmc_save_snapshot", rc);
    printf("# acceptance %.6f (accepted %lld / trials %lld, energy-evaluated %lld)\n",
           total.trials ? (double)total.accepted / (double)total.trials : 0.0, (long long)total.accepted,
           (long long)total.trials, (long long)total.evaluated);
    if (seconds > 0)
        printf("# device time %.6f s, %.3e trial-moves/s\n", seconds, (double)total.trials / seconds);
    pmc_destroy(ctx);
    return 0;
}
