// icp_bench.cpp — the reference's google-benchmark cases (src/bench.cc:391-445), GPU side, on
// this engine through the C ABI (include/icp_capi.h).  Same case names, same inputs and the
// same per-iteration work; reports real time per iteration and the `frame_rate` counter
// (iterations / s, bench.cc:78 ...).  The six cpu_* cases time the reference's CPU path,
// which here is the oracle (test infrastructure): bench.py times those in its cpu_baseline
// leg.
//
//   icp-bench [--ref PATH] [--scene PATH] [--min-time SECONDS] [--json] [--cold] [--only NAME]
//
// Inputs follow the reference's parameter functions (bench.cc:241-389), quirks included:
//  * gpu_find_alignment, gpu_err_compute*: Y = Matrix::Zero (bench.cc:270-276, 378-388);
//  * gpu_err_compute / _alignment: sr = (bool in_place) * r, i.e. 0 and I (gpu.hh:64-71);
//  * opti_gpu_closest_matrix: compute_Y_w_opti(p, m, y) with the scene in the model slot
//    (bench.cc:186, signature gpu.hh:110);
//  * *_loop: a fresh registration per iteration, max_iter 20, threshold 1e-5 (bench.cc:65-102).
// Differences by design: the model stays resident in the context, where the
// reference re-uploads it on every call; `--cold` adds icp_set_model to every loop iteration.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/icp_capi.h"

namespace {

struct Cloud {
    std::vector<double> xyz;
    size_t n = 0;
};

bool load(const char *path, Cloud &c)
{
    double *p = nullptr;
    size_t n = 0;
    if (icp_load_matrix(path, &p, &n) != ICP_OK) return false;
    c.xyz.assign(p, p + 3 * n);
    c.n = n;
    icp_free(p);
    return true;
}

void check(icp_ctx *ctx, int rc, const char *what)
{
    if (rc != ICP_OK) {
        std::fprintf(stderr, "[icp-bench] %s failed: %s (%s)\n", what, icp_strerror(rc),
                     ctx ? icp_last_error(ctx) : "");
        std::exit(1);
    }
}

struct Result {
    std::string name;
    double ms = 0;
    long iterations = 0;
};

// google-benchmark style: run until min_time has elapsed (at least one timed iteration)
std::string g_only; // --only: run just this case

Result run_case(const std::string &name, double min_time, const std::function<void()> &body)
{
    if (!g_only.empty() && name != g_only) return {name, 0.0, 0};
    body(); // warm-up (first-launch costs)
    long it = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    do {
        body();
        ++it;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < min_time);
    return {name, el * 1e3 / (double)it, it};
}

} // namespace

int main(int argc, char **argv)
{
    std::string ref = "data_students/cow_ref.txt", scene = "data_students/cow_tr1.txt";
    double min_time = 0.5;
    bool json = false, cold = false;
    std::string only;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--ref" && i + 1 < argc) ref = argv[++i];
        else if (a == "--scene" && i + 1 < argc) scene = argv[++i];
        else if (a == "--min-time" && i + 1 < argc) min_time = std::atof(argv[++i]);
        else if (a == "--json") json = true;
        else if (a == "--cold") cold = true;
        else if (a == "--only" && i + 1 < argc) only = argv[++i];
        else {
            std::fprintf(stderr, "usage: icp-bench [--ref PATH] [--scene PATH] [--min-time S] [--json] [--cold]\n");
            return 2;
        }
    }
    g_only = only;
    Cloud m, p;
    if (!load(ref.c_str(), m) || !load(scene.c_str(), p)) {
        std::fprintf(stderr, "[icp-bench] cannot read %s / %s\n", ref.c_str(), scene.c_str());
        return 2;
    }
    icp_ctx *ctx = nullptr;
    check(nullptr, icp_ctx_create(0, ICP_NN_CERTIFIED, &ctx), "icp_ctx_create");
    const size_t np = p.n;
    std::vector<double> Y(3 * np, 0.0), Yz(3 * np, 0.0), tmp(3 * np), cent(3 * np);
    std::vector<Result> out;

    // naive_gpu_closest_matrix: GPU::ICP::compute_y_naive (gpu.cc:6-15), one NN call per point
    check(ctx, icp_set_model(ctx, m.xyz.data(), m.n), "icp_set_model");
    out.push_back(run_case("naive_gpu_closest_matrix", min_time, [&] {
        for (size_t j = 0; j < np; ++j)
            check(ctx, icp_closest_matrix(ctx, &p.xyz[3 * j], 1, &Y[3 * j], nullptr), "closest (1 point)");
    }));

    // opti_gpu_closest_matrix: compute_Y_w_opti(params.p, params.m, params.y) — the scene is
    // passed as the model argument (bench.cc:186)
    check(ctx, icp_set_model(ctx, p.xyz.data(), p.n), "icp_set_model");
    out.push_back(run_case("opti_gpu_closest_matrix", min_time, [&] {
        check(ctx, icp_closest_matrix(ctx, m.xyz.data(), m.n, tmp.data(), nullptr), "closest_matrix");
    }));
    check(ctx, icp_set_model(ctx, m.xyz.data(), m.n), "icp_set_model");

    // gpu_find_alignment: icp.find_alignment(Y) with Y = 0 (bench.cc:378-388)
    out.push_back(run_case("gpu_find_alignment", min_time, [&] {
        double s, R[9], t[3], err;
        check(ctx, icp_find_alignment(ctx, p.xyz.data(), Yz.data(), np, &s, R, t, &err), "find_alignment");
    }));

    // gpu_compute_centroid: means + substract_col_w of new_p and of its correspondences
    check(ctx, icp_closest_matrix(ctx, p.xyz.data(), np, Y.data(), nullptr), "closest_matrix");
    out.push_back(run_case("gpu_compute_centroid", min_time, [&] {
        double mu[3];
        check(ctx, icp_compute_centroid(ctx, p.xyz.data(), np, mu, cent.data()), "compute_centroid");
        check(ctx, icp_compute_centroid(ctx, Y.data(), np, mu, cent.data()), "compute_centroid");
    }));

    // gpu_err_compute(_alignment): compute_err_w(Y = 0, p, in_place, sr = in_place * r, t = 0)
    const double zero9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, eye9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double t0[3] = {0, 0, 0};
    out.push_back(run_case("gpu_err_compute", min_time, [&] {
        double err;
        std::memcpy(tmp.data(), p.xyz.data(), sizeof(double) * 3 * np); // GPU::Matrix p_ = params.p
        check(ctx, icp_err_compute(ctx, Yz.data(), tmp.data(), np, 0, zero9, t0, &err), "err_compute");
    }));
    out.push_back(run_case("gpu_err_compute_alignment", min_time, [&] {
        double err;
        std::memcpy(tmp.data(), p.xyz.data(), sizeof(double) * 3 * np);
        check(ctx, icp_err_compute(ctx, Yz.data(), tmp.data(), np, 1, eye9, t0, &err), "err_compute");
    }));

    // naive_gpu_loop: GPU::ICP::find_corresponding_naive (gpu.cc:17-49) on the wrappers
    int naive_iters = 0;
    out.push_back(run_case("naive_gpu_loop", min_time, [&] {
        std::memcpy(tmp.data(), p.xyz.data(), sizeof(double) * 3 * np); // new_p = p
        for (int i = 0; i < 20; ++i) {
            for (size_t j = 0; j < np; ++j)
                check(ctx, icp_closest_matrix(ctx, &tmp[3 * j], 1, &Y[3 * j], nullptr), "closest (1 point)");
            double s, R[9], t[3], err, e2;
            check(ctx, icp_find_alignment(ctx, tmp.data(), Y.data(), np, &s, R, t, &err), "find_alignment");
            double sR[9];
            for (int k = 0; k < 9; ++k) sR[k] = s * R[k];
            check(ctx, icp_err_compute(ctx, Y.data(), tmp.data(), np, 1, sR, t, &e2), "err_compute");
            naive_iters = i + 1;
            if ((err + e2) / (double)np < 1e-5) break;
        }
    }));

    // opti_gpu_loop: GPU::ICP::find_corresponding_opti (gpu.cc:52-83), a fresh ICP per iteration
    icp_result res{};
    out.push_back(run_case(cold ? "opti_gpu_loop_cold" : "opti_gpu_loop", min_time, [&] {
        if (cold) check(ctx, icp_set_model(ctx, m.xyz.data(), m.n), "icp_set_model");
        check(ctx, icp_set_scene(ctx, p.xyz.data(), np, np), "icp_set_scene");
        check(ctx, icp_run(ctx, 20, 1e-5, nullptr, &res), "icp_run");
    }));
    icp_ctx_destroy(ctx);

    if (json) {
        std::printf("{\"ref\": \"%s\", \"scene\": \"%s\", \"opti_iterations\": %d, \"naive_iterations\": %d, \"cases\": {",
                    ref.c_str(), scene.c_str(), res.iterations, naive_iters);
        bool first = true;
        for (size_t i = 0; i < out.size(); ++i) {
            if (!out[i].iterations) continue;
            std::printf("%s\"%s\": {\"ms\": %.6g, \"iterations\": %ld, \"frame_rate\": %.6g}", first ? "" : ", ",
                        out[i].name.c_str(), out[i].ms, out[i].iterations, 1e3 / out[i].ms);
            first = false;
        }
        std::printf("}}\n");
    } else {
        std::printf("%-40s %14s %12s %s\n", "Benchmark", "Time", "Iterations", "UserCounters...");
        for (const auto &r : out)
            if (r.iterations)
                std::printf("%-40s %11.4g ms %12ld frame_rate=%.6g/s\n", (r.name + "/real_time").c_str(), r.ms,
                        r.iterations, 1e3 / r.ms);
    }
    return 0;
}
