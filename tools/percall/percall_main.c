/*
 * percall_main.c -- driver for liquid-dsp's own per-call benchmark bodies.
 *
 * tools/build_ref_benches.sh compiles the reference's benchmark sources
 * (src/{filter,dotprod,multichannel,buffer}/bench/ *_benchmark.c) unchanged
 * against include/liquid.h and libliquid_mi355x.so, with getrusage()
 * renamed to lqb_getrusage() below, and links them with this file.  The
 * reference harness (bench/bench.c:357-391) times those bodies with
 * getrusage CPU time; a GPU library spends most of a call waiting on the
 * device, so here the same start/finish hooks record CLOCK_MONOTONIC wall
 * time instead.  The trial count doubles until a run lasts --runtime
 * seconds (bench.c:361-381); the rate is trials / second, a trial being
 * what the reference counts (one output sample, one dot product, one
 * channelizer call ... BASELINE.md section 2).
 *
 *   percall [--runtime S] [--base N] name...   one JSON line per benchmark
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

typedef void (*bench_fn)(struct rusage *, struct rusage *, unsigned long int *);

#include "bench_table.h" /* generated: LQB_DECLS and LQB_TABLE */

LQB_DECLS

static const struct {
    const char *name;
    bench_fn fn;
} table[] = {LQB_TABLE};

int lqb_getrusage(int who, struct rusage *u)
{
    (void)who;
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    memset(u, 0, sizeof(*u));
    u->ru_utime.tv_sec = t.tv_sec;
    u->ru_utime.tv_usec = t.tv_nsec / 1000;
    return 0;
}

static double elapsed(const struct rusage *a, const struct rusage *b)
{
    return (double)(b->ru_utime.tv_sec - a->ru_utime.tv_sec) + 1e-6 * (double)(b->ru_utime.tv_usec - a->ru_utime.tv_usec);
}

int main(int argc, char **argv)
{
    double runtime = 0.25;
    unsigned long base = 256;
    int i = 1;
    for (; i < argc && !strncmp(argv[i], "--", 2); i += 2) {
        if (i + 1 >= argc) break;
        if (!strcmp(argv[i], "--runtime")) runtime = atof(argv[i + 1]);
        else if (!strcmp(argv[i], "--base")) base = strtoul(argv[i + 1], NULL, 10);
    }
    const int nt = (int)(sizeof(table) / sizeof(table[0]));
    for (; i < argc; i++) {
        int k = 0;
        while (k < nt && strcmp(table[k].name, argv[i])) k++;
        if (k == nt) {
            printf("{\"name\": \"%s\", \"error\": \"not built\"}\n", argv[i]);
            continue;
        }
        unsigned long n = base, trials = 0;
        double t = 0.0;
        struct rusage s, f;
        for (int attempt = 0; attempt < 24; attempt++, n *= 2) {
            trials = n;
            table[k].fn(&s, &f, &trials);
            t = elapsed(&s, &f);
            if (t >= runtime) break;
        }
        printf("{\"name\": \"%s\", \"trials\": %lu, \"seconds\": %.6f, \"trials_per_s\": %.6g, \"us_per_trial\": %.4f}\n",
               argv[i], trials, t, t > 0 ? (double)trials / t : 0.0, t > 0 ? 1e6 * t / (double)trials : 0.0);
        fflush(stdout);
    }
    return 0;
}
