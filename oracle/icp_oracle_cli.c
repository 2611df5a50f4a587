/*
 * icp_oracle_cli.c — TEST INFRASTRUCTURE ONLY.
 * Restates the reference CPU CLI src/main.cc:6-25 (`icp <ref> <scene> <iters>`) on
 * top of the oracle, with the reference's stderr lines (cpu.cc:61,74; load.cc:8,19,80)
 * and output.txt.  Extra flags (after the 3 positionals) for test use only:
 *   --allow-unequal   run even if np != nm (reference exits, cpu.cc:44-47)
 *   --nn-sqrt         faithful cpu.cc sqrt(pow()) distances (default: squared)
 *   --threshold X     override cpu.hh:113's 1e-5
 *   --out PATH        output file (default ./output.txt, load.cc:71)
 */
#include "icp_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv)
{
    if (argc < 4) {
        printf("Usage: ./icp [path_to_ref_cloud] [path_to_transform_cloud] [nb_iter]\n");
        return -1;
    }
    int max_iter = atoi(argv[3]);
    int allow_unequal = 0, nn_mode = ORACLE_NN_SQUARED;
    double threshold = 1e-5;
    const char *out = "output.txt";
    for (int a = 4; a < argc; ++a) {
        if (!strcmp(argv[a], "--allow-unequal")) allow_unequal = 1;
        else if (!strcmp(argv[a], "--nn-sqrt")) nn_mode = ORACLE_NN_CPU_SQRT;
        else if (!strcmp(argv[a], "--threshold") && a + 1 < argc) threshold = atof(argv[++a]);
        else if (!strcmp(argv[a], "--out") && a + 1 < argc) out = argv[++a];
    }
    size_t nm = 0, np = 0;
    fprintf(stderr, "[load] opening %s\n", argv[1]);
    double *m = oracle_load_matrix(argv[1], &nm);
    if (!m) { fprintf(stderr, "[load] %s could not be opened\n", argv[1]); return 2; }
    fprintf(stderr, "[load] loading file into matrix\n");
    fprintf(stderr, "[load] opening %s\n", argv[2]);
    double *p = oracle_load_matrix(argv[2], &np);
    if (!p) { fprintf(stderr, "[load] %s could not be opened\n", argv[2]); return 2; }
    fprintf(stderr, "[load] loading file into matrix\n");

    if (np != nm && !allow_unequal) {
        fprintf(stderr, "[error] Point sets need to have the same number of points.\n");
        return 255;
    }
    if (np < 4) {
        fprintf(stderr, "[error] Need at least 4 point pairs\n");
        return 255;
    }
    double *errs = (double *)calloc(max_iter > 0 ? (size_t)max_iter : 1, sizeof(double));
    oracle_trace tr = {errs, NULL, NULL, NULL, NULL};
    int it = oracle_icp(m, nm, p, np, max_iter, threshold, nn_mode, allow_unequal, &tr);
    for (int i = 0; i < it; ++i)
        fprintf(stderr, "[ICP] iteration number %d | error value = %g\n", i, errs[i]);
    oracle_write_matrix(out, p, np);
    fprintf(stderr, "[output] output file \"%s\" was generated.\n", out);
    free(errs);
    free(m);
    free(p);
    return 0;
}
