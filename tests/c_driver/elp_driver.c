/*
 * elp_driver.c -- a plain C caller of libeasylp_hip.so, the way the R .Call
 * shim drives it: no Python, no torch, so the library runs on
 * /opt/rocm's HIP runtime through its RUNPATH, A comes from host memory
 * (elp_load_dense), and with `ngpu P` one process drives P rank handles.
 * Test infrastructure (tests/test_gpu_c_driver.py builds and runs it).
 *
 *   elp_driver INPUT [ngpu P] [trace CAP]
 *
 * INPUT (whitespace-separated text, "inf" / "-inf" accepted):
 *   count
 *   per LP:  m n maximize
 *            A (m*n values, column-major, R's layout)   dir (m)   rhs (m)
 *            obj (n)   lo (n)   up (n)
 * Output per LP (stdout):
 *   lp <i> rc <rc> status <s> objective <%.17g> iterations <it> exchange <e>
 *   x <n values>
 *   basis <m ids>
 *   trace <count> <pairs...>            (with `trace CAP`)
 * plus one line "runtime <path of the libamdhip64 mapped into this process>".
 * Mirrors the seam R/class.R:260-278 (make.lp ... solve ... get.variables).
 */
#define _GNU_SOURCE
#include <link.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/easylp_hip.h"

static int hip_path(struct dl_phdr_info* info, size_t size, void* data) {
    (void)size;
    if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64")) {
        snprintf((char*)data, 1024, "%s", info->dlpi_name);
        return 1;
    }
    return 0;
}

static int rd(FILE* f, double* v, long long cnt) {
    for (long long i = 0; i < cnt; ++i) {
        char tok[64];
        if (fscanf(f, "%63s", tok) != 1) return -1;
        v[i] = strtod(tok, NULL);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s INPUT [ngpu P] [trace CAP]\n", argv[0]);
        return 2;
    }
    int ngpu = 1;
    long long cap = 0;
    for (int a = 2; a + 1 < argc; a += 2) {
        if (!strcmp(argv[a], "ngpu")) ngpu = atoi(argv[a + 1]);
        else if (!strcmp(argv[a], "trace")) cap = atoll(argv[a + 1]);
    }
    FILE* f = fopen(argv[1], "r");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    int count = 0;
    if (fscanf(f, "%d", &count) != 1) return 2;
    elp_control ctl;
    elp_default_control(&ctl);
    ctl.ngpu = ngpu;
    int bad = 0;
    for (int lp = 0; lp < count; ++lp) {
        long long m, n;
        int mx;
        if (fscanf(f, "%lld %lld %d", &m, &n, &mx) != 3) return 2;
        double* A = malloc(sizeof(double) * (size_t)(m * n + 1));
        double* rhs = malloc(sizeof(double) * (size_t)(m + 1));
        double* dird = malloc(sizeof(double) * (size_t)(m + 1));
        int32_t* dir = malloc(sizeof(int32_t) * (size_t)(m + 1));
        double* obj = malloc(sizeof(double) * (size_t)n);
        double* lo = malloc(sizeof(double) * (size_t)n);
        double* up = malloc(sizeof(double) * (size_t)n);
        double* x = malloc(sizeof(double) * (size_t)n);
        int64_t* basis = malloc(sizeof(int64_t) * (size_t)(m + 1));
        if (rd(f, A, m * n) || rd(f, dird, m) || rd(f, rhs, m) || rd(f, obj, n) || rd(f, lo, n) || rd(f, up, n))
            return 2;
        for (long long i = 0; i < m; ++i) dir[i] = (int32_t)dird[i];
        elp_handle* h = NULL;
        int32_t st = -1;
        double z = 0.0;
        ctl.ngpu = ngpu < n ? ngpu : (int)n; /* a rank prices at least one column */
        int rc = elp_create(&h, m, n, &ctl);
        if (!rc && cap > 0) rc = elp_set_trace(h, cap);
        if (!rc) rc = elp_load_dense(h, A, dir, rhs, obj, lo, up, mx);
        if (!rc) rc = elp_solve(h, &st);
        if (!rc) rc = elp_get_solution(h, &z, x, NULL, basis);
        elp_stats s;
        memset(&s, 0, sizeof(s));
        if (!rc) rc = elp_get_stats(h, &s);
        if (rc) {
            fprintf(stderr, "lp %d: rc %d: %s\n", lp, rc, elp_last_error());
            bad = 1;
        }
        printf("lp %d rc %d status %d objective %.17g iterations %lld exchange %d\n", lp, rc, st, z,
               (long long)s.iterations, s.exchange);
        printf("x");
        for (long long j = 0; j < n; ++j) printf(" %.17g", x[j]);
        printf("\nbasis");
        for (long long i = 0; i < m; ++i) printf(" %lld", (long long)basis[i]);
        printf("\n");
        if (cap > 0 && !rc) {
            int64_t* pairs = malloc(sizeof(int64_t) * (size_t)(2 * cap));
            int64_t cnt = 0;
            if (elp_get_trace(h, pairs, cap, &cnt) == 0) {
                printf("trace %lld", (long long)cnt);
                for (int64_t t = 0; t < 2 * cnt; ++t) printf(" %lld", (long long)pairs[t]);
                printf("\n");
            }
            free(pairs);
        }
        if (h) elp_destroy(h);
        free(A), free(rhs), free(dird), free(dir), free(obj), free(lo), free(up), free(x), free(basis);
    }
    char path[1024] = "none";
    dl_iterate_phdr(hip_path, path);
    printf("runtime %s\n", path);
    fclose(f);
    return bad;
}
