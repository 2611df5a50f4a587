// icp_cli.cpp — `icp-gpu` / `icp` command line (src/GPU/main.cc:3-21, src/main.cc:6-25).
//
//   icp-gpu <path_to_ref_cloud> <path_to_transform_cloud> <nb_iter> [options]
//
// Same positional contract, stderr lines ([load] / [ICP] / [output]), ./output.txt and
// exit codes as the reference.  Both binaries run the HIP engine (there is no CPU
// fallback in the product).  `icp` keeps the reference CPU path's NN rule (src/main.cc ->
// cpu.cc:17-22: first minimum of sqrt(pow() sums), ICP_NN_RULE_CPU_SQRT) and `icp-gpu` the GPU
// path's (compute.cu:112-117: squared distances); they differ only at near ties.
// Options (after the positionals):
//   --rule cpu|squared override the binary's NN rule
//   --allow-unequal    run even when the clouds differ in size (reference: exit 255)
//   --nn fp64|certified  NN arithmetic (default certified; identical results)
//   --threshold X      convergence threshold (default 1e-5, src/cpu.hh:113)
//   --out PATH         output file (default output.txt, src/load.cc:71)
//   --device D         HIP device ordinal (default 0)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/icp_capi.h"

static double *load_or_exit(const char *path, size_t *n)
{
    std::fprintf(stderr, "[load] opening %s\n", path); // load.cc:8
    double *xyz = nullptr;
    if (icp_load_matrix(path, &xyz, n) != ICP_OK) {
        std::fprintf(stderr, "[load] %s could not be opened\n", path); // load.cc:11-13
        std::exit(2);
    }
    std::fprintf(stderr, "[load] loading file into matrix\n"); // load.cc:19
    return xyz;
}

int main(int argc, char **argv)
{
    const char *prog = std::strrchr(argv[0], '/') ? std::strrchr(argv[0], '/') + 1 : argv[0];
    if (argc < 4) { // main.cc:5-8
        std::printf("Usage: ./%s [path_to_ref_cloud] [path_to_transform_cloud] [nb_iter]\n", prog);
        return -1;
    }
    const int max_iter = std::atoi(argv[3]);
    bool allow_unequal = false;
    int nn_mode = ICP_NN_CERTIFIED, device = 0;
    int rule = std::strcmp(prog, "icp") == 0 ? ICP_NN_RULE_CPU_SQRT : ICP_NN_RULE_SQUARED;
    double threshold = 1e-5;
    const char *out = "output.txt";
    for (int a = 4; a < argc; ++a) {
        if (!std::strcmp(argv[a], "--allow-unequal")) allow_unequal = true;
        else if (!std::strcmp(argv[a], "--nn") && a + 1 < argc) {
            ++a;
            nn_mode = !std::strcmp(argv[a], "fp64") ? ICP_NN_FP64 : ICP_NN_CERTIFIED;
        } else if (!std::strcmp(argv[a], "--rule") && a + 1 < argc) {
            ++a;
            rule = !std::strcmp(argv[a], "cpu") ? ICP_NN_RULE_CPU_SQRT : ICP_NN_RULE_SQUARED;
        } else if (!std::strcmp(argv[a], "--threshold") && a + 1 < argc) threshold = std::atof(argv[++a]);
        else if (!std::strcmp(argv[a], "--out") && a + 1 < argc) out = argv[++a];
        else if (!std::strcmp(argv[a], "--device") && a + 1 < argc) device = std::atoi(argv[++a]);
        else {
            std::fprintf(stderr, "[error] unknown option %s\n", argv[a]);
            return -1;
        }
    }

    size_t nm = 0, np = 0;
    double *m = load_or_exit(argv[1], &nm);
    double *p = load_or_exit(argv[2], &np);

    // alignement_check (cpu.cc:42-53 / gpu.cc:54-62): message + exit(-1)
    if (np != nm && !allow_unequal) {
        std::fprintf(stderr, "[error] Point sets need to have the same number of points.\n");
        return -1;
    }
    if (np < 4) {
        std::fprintf(stderr, "[error] Need at least 4 point pairs\n");
        return -1;
    }

    icp_ctx *ctx = nullptr;
    int rc = icp_ctx_create(device, nn_mode, &ctx);
    if (rc != ICP_OK) {
        std::fprintf(stderr, "[error] %s\n", icp_strerror(rc));
        return 3;
    }
    icp_set_allow_unequal(ctx, allow_unequal ? 1 : 0);
    icp_set_nn_rule(ctx, rule);
    if ((rc = icp_set_model(ctx, m, nm)) != ICP_OK || (rc = icp_set_scene(ctx, p, np, np)) != ICP_OK) {
        std::fprintf(stderr, "[error] %s: %s\n", icp_strerror(rc), icp_last_error(ctx));
        return 3;
    }
    double *errs = (double *)std::calloc(max_iter > 0 ? (size_t)max_iter : 1, sizeof(double));
    icp_result res{};
    // each iteration's line as it ends (gpu.cc:65,77), from the engine's progress callback
    icp_set_progress(
        ctx, [](int i, double e, void *) { std::fprintf(stderr, "[ICP] iteration number %d | error value = %g\n", i, e); },
        nullptr);
    rc = icp_run(ctx, max_iter, threshold, errs, &res);
    if (rc != ICP_OK) {
        std::fprintf(stderr, "[error] %s: %s\n", icp_strerror(rc), icp_last_error(ctx));
        return 3;
    }
    if ((rc = icp_get_scene(ctx, p)) != ICP_OK) {
        std::fprintf(stderr, "[error] %s: %s\n", icp_strerror(rc), icp_last_error(ctx));
        return 3;
    }
    if (icp_write_matrix(out, p, np) != ICP_OK) { // load.cc:68-81
        std::fprintf(stderr, "[error] cannot write %s\n", out);
        return 2;
    }
    std::fprintf(stderr, "[output] output file \"%s\" was generated.\n", out);
    icp_ctx_destroy(ctx);
    std::free(errs);
    icp_free(m);
    icp_free(p);
    return 0;
}
