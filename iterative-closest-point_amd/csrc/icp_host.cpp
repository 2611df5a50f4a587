// icp_host.cpp — host-side pieces of the ICP engine that need no device:
// Horn's closed-form alignment solve, scene sharding, the synthetic cloud generator
// and CSV point-cloud I/O.  Part of libicp_hip.so (product code, not the oracle).
//
// Reference: src/GPU/gpu.cc:95-151 (find_alignment, host half), gpu.cc:85-93
// (max_element_index), src/load.cc:3-97 (I/O).
#include "icp_internal.h"
#include "icp_horn.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace icp {


void shard_range(size_t n, int rank, int world, size_t *begin, size_t *count)
{
    const size_t base = n / (size_t)world, rem = n % (size_t)world;
    const size_t r = (size_t)rank;
    *begin = r * base + (r < rem ? r : rem);
    *count = base + (r < rem ? 1 : 0);
}

// ---- CSV point-cloud I/O (src/load.cc:3-97) ---------------------------------------------
// Row semantics of load.cc:26-27: sscanf(line, "%lf,%lf,%lf") into zero-initialised x, y, z.
// glibc's %lf is greedier than strtod: it consumes "1e" or "1e+" (an exponent marker with no
// digits) and converts the consumed text, so "1e,2,3" is (1, 2, 3).  Rows the fast path
// below does not fully cover go through that very call.
static void parse_row_sscanf(const char *line, double out[3])
{
    double x = 0., y = 0., z = 0.;
    std::sscanf(line, "%lf,%lf,%lf", &x, &y, &z);
    out[0] = x;
    out[1] = y;
    out[2] = z;
}

// Clinger's exact fast path: [-]digits[.digits][(e|E)[+-]digits] with a decimal mantissa
// m <= 2^53 and |exponent| <= 22 is m * 10^e (or m / 10^-e): one correctly rounded operation
// on exact operands, i.e. the same double strtod (and so %lf) returns.  Anything else
// (whitespace, '+', hex, inf/nan, long mantissas, huge exponents, a bare exponent marker)
// -> false, and the row goes through sscanf.
static bool parse_number_fast(const char *s, const char *end, double &v, const char *&stop)
{
    static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const char *p = s;
    bool neg = false;
    if (p < end && *p == '-') {
        neg = true;
        ++p;
    }
    uint64_t m = 0;
    int exp10 = 0;
    bool any = false;
    const uint64_t kMax = (uint64_t)1 << 53;
    const char *int_start = p;
    while (p < end && *p >= '0' && *p <= '9') {
        m = m * 10 + (uint64_t)(*p - '0');
        if (m > kMax) return false;
        ++p;
        any = true;
    }
    if (p < end && (*p == 'x' || *p == 'X') && p - int_start == 1 && *int_start == '0') return false; // hex
    if (p < end && *p == '.') {
        ++p;
        while (p < end && *p >= '0' && *p <= '9') {
            m = m * 10 + (uint64_t)(*p - '0');
            if (m > kMax) return false;
            --exp10;
            ++p;
            any = true;
        }
    }
    if (!any) return false;
    if (p < end && (*p == 'e' || *p == 'E')) {
        const char *q = p + 1;
        bool eneg = false;
        if (q < end && (*q == '+' || *q == '-')) {
            eneg = *q == '-';
            ++q;
        }
        if (!(q < end && *q >= '0' && *q <= '9')) return false; // "1e", "1e+": sscanf's own rule
        {
            int ex = 0;
            while (q < end && *q >= '0' && *q <= '9') {
                if (ex > 10000) return false;
                ex = ex * 10 + (*q - '0');
                ++q;
            }
            exp10 += eneg ? -ex : ex;
            p = q;
        }
    }
    if (exp10 < -22 || exp10 > 22) return false;
    const double dm = (double)m; // exact: m <= 2^53
    v = exp10 >= 0 ? dm * kPow10[exp10] : dm / kPow10[-exp10];
    if (neg) v = -v;
    stop = p;
    return true;
}

// one row [s, end) (end = its '\n' or the end of the file)
static void parse_row(const char *s, const char *end, double out[3])
{
    double v[3] = {0, 0, 0};
    const char *p = s;
    for (int k = 0; k < 3; ++k) {
        const char *e = nullptr;
        if (!parse_number_fast(p, end, v[k], e)) { // any other form: the reference's own call
            const std::string line(s, (size_t)(end - s));
            parse_row_sscanf(line.c_str(), out);
            return;
        }
        out[k] = v[k];
        if (k < 2) {
            if (e >= end || *e != ',') return;
            p = e + 1;
        }
    }
}

static unsigned io_threads(size_t bytes)
{
    unsigned t = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("ICP_IO_THREADS")) t = (unsigned)std::atoi(e);
    t = std::max(1u, std::min(t, 16u));
    return (unsigned)std::max<size_t>(1, std::min<size_t>(t, bytes / (1 << 20) + 1)); // >= 1 MiB each
}

int load_matrix(const char *path, std::vector<double> &xyz, size_t *n_out)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) return ICP_E_IO;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<char> buf(sz > 0 ? (size_t)sz + 1 : 1, '\0');
    const size_t got = sz > 0 ? std::fread(buf.data(), 1, (size_t)sz, f) : 0;
    std::fclose(f);
    buf[got] = '\0';
    const char *base = buf.data(), *end = base + got;
    // chunks at arbitrary byte offsets; a '\n' at offset q starts row (#'\n' before q), the
    // header being line 0 (load.cc:21)
    const unsigned T = io_threads(got);
    std::vector<size_t> cut(T + 1), nl(T + 1, 0);
    for (unsigned t = 0; t <= T; ++t) cut[t] = got * t / T;
    auto count = [&](unsigned t) {
        size_t c = 0;
        for (const char *p = base + cut[t], *e = base + cut[t + 1];
             (p = (const char *)std::memchr(p, '\n', (size_t)(e - p))) != nullptr; ++p)
            ++c;
        nl[t + 1] = c;
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; ++t) pool.emplace_back(count, t);
    count(0);
    for (auto &th : pool) th.join();
    pool.clear();
    for (unsigned t = 0; t < T; ++t) nl[t + 1] += nl[t];
    // load.cc:15-17: getline() count minus the header
    const size_t lines = nl[T] + ((got && buf[got - 1] != '\n') ? 1 : 0);
    const size_t n = lines > 0 ? lines - 1 : 0;
    xyz.assign(3 * n, 0.0);
    auto parse = [&](unsigned t) {
        size_t row = nl[t];
        for (const char *p = base + cut[t], *e = base + cut[t + 1];
             (p = (const char *)std::memchr(p, '\n', (size_t)(e - p))) != nullptr; ++p, ++row) {
            if (row >= n) break;
            const char *s = p + 1;
            const char *le = (const char *)std::memchr(s, '\n', (size_t)(end - s));
            parse_row(s, le ? le : end, &xyz[3 * row]);
        }
    };
    for (unsigned t = 1; t < T; ++t) pool.emplace_back(parse, t);
    parse(0);
    for (auto &th : pool) th.join();
    *n_out = n;
    return ICP_OK;
}

// load.cc:68-81: header, then `os << x << ',' << y << ',' << z << std::endl` with the default
// stream format (precision 6, %g).  Rows are formatted in parallel, written in order.
int write_matrix(const char *path, const double *xyz, size_t n)
{
    FILE *f = std::fopen(path, "wb");
    if (!f) return ICP_E_IO;
    std::fputs("Points_0,Points_1,Points_2\n", f);
    const unsigned T = io_threads(n * 40);
    std::vector<std::string> part(T);
    auto fmt = [&](unsigned t) {
        const size_t j0 = n * t / T, j1 = n * (t + 1) / T;
        std::string &o = part[t];
        o.reserve((j1 - j0) * 40);
        char line[128];
        for (size_t j = j0; j < j1; ++j) {
            // std::to_chars(general, 6) is specified as printf("%.6g") in the C locale (the
            // stream default); Ryu-based, and without glibc printf's shared state
            char *c = line;
            for (int k = 0; k < 3; ++k) {
                c = std::to_chars(c, line + sizeof(line), xyz[3 * j + k], std::chars_format::general, 6).ptr;
                *c++ = k < 2 ? ',' : '\n';
            }
            o.append(line, (size_t)(c - line));
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; ++t) pool.emplace_back(fmt, t);
    fmt(0);
    for (auto &th : pool) th.join();
    bool ok = true;
    for (const auto &o : part) ok = ok && std::fwrite(o.data(), 1, o.size(), f) == o.size();
    ok = (std::fclose(f) == 0) && ok;
    return ok ? ICP_OK : ICP_E_IO;
}

void synthetic_pair(uint64_t seed, size_t n, double angle_deg, const double axis_in[3],
                    const double tr[3], double *model, double *scene)
{
    std::mt19937_64 gen(seed);
    for (size_t i = 0; i < 3 * n; ++i) {
        // 53 random bits -> [0,1) -> [-1,1), rounded to an fp32-representable double
        const double u = (double)(gen() >> 11) * 0x1.0p-53;
        model[i] = (double)(float)(2.0 * u - 1.0);
    }
    double ax[3] = {axis_in[0], axis_in[1], axis_in[2]};
    const double nrm = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    for (double &a : ax) a /= nrm;
    const double th = angle_deg * M_PI / 180.0, c = std::cos(th), s = std::sin(th), C = 1.0 - c;
    const double R[9] = {c + ax[0] * ax[0] * C,         ax[0] * ax[1] * C - ax[2] * s, ax[0] * ax[2] * C + ax[1] * s,
                         ax[1] * ax[0] * C + ax[2] * s, c + ax[1] * ax[1] * C,         ax[1] * ax[2] * C - ax[0] * s,
                         ax[2] * ax[0] * C - ax[1] * s, ax[2] * ax[1] * C + ax[0] * s, c + ax[2] * ax[2] * C};
    for (size_t j = 0; j < n; ++j) {
        double q[3];
        matvec3(R, model + 3 * j, q);
        for (int k = 0; k < 3; ++k) scene[3 * j + k] = (double)(float)(q[k] + tr[k]);
    }
}

} // namespace icp

// ---- C-ABI wrappers for the host-only entry points ------------------------------
extern "C" {

int icp_horn_solve(const double S[9], const double mu_p[3], const double mu_y[3], double d_caps,
                   double sp, double *s, double R[9], double t[3])
{
    if (!S || !mu_p || !mu_y || !s || !R || !t) return ICP_E_ARG;
    icp::horn_solve(S, mu_p, mu_y, d_caps, sp, s, R, t);
    return ICP_OK;
}

int icp_max_element_index(const double ev[4])
{
    // gpu.cc:85-93 as written: `max` is never updated, so this is the LAST i in 1..3
    // with ev[i] > ev[0] (not the argmax in general).
    int index = 0;
    const double max = ev[0];
    for (int i = 1; i < 4; ++i)
        if (ev[i] > max) index = i;
    return index;
}

int icp_shard_range(size_t n_total, int rank, int world_size, size_t *begin, size_t *count)
{
    if (world_size < 1 || rank < 0 || rank >= world_size || !begin || !count) return ICP_E_ARG;
    icp::shard_range(n_total, rank, world_size, begin, count);
    return ICP_OK;
}

int icp_synthetic_pair(uint64_t seed, size_t n, double angle_deg, const double axis[3],
                       const double t[3], double *model_xyz_out, double *scene_xyz_out)
{
    if (!axis || !t || !model_xyz_out || !scene_xyz_out) return ICP_E_ARG;
    icp::synthetic_pair(seed, n, angle_deg, axis, t, model_xyz_out, scene_xyz_out);
    return ICP_OK;
}

int icp_load_matrix(const char *path, double **xyz_out, size_t *n_out)
{
    if (!path || !xyz_out || !n_out) return ICP_E_ARG;
    std::vector<double> v;
    size_t n = 0;
    int rc = icp::load_matrix(path, v, &n);
    if (rc != ICP_OK) return rc;
    double *out = (double *)std::malloc(sizeof(double) * (v.size() ? v.size() : 1));
    if (!out) return ICP_E_ARG;
    if (!v.empty()) std::memcpy(out, v.data(), sizeof(double) * v.size());
    *xyz_out = out;
    *n_out = n;
    return ICP_OK;
}

int icp_write_matrix(const char *path, const double *xyz, size_t n)
{
    if (!path || (!xyz && n)) return ICP_E_ARG;
    return icp::write_matrix(path, xyz, n);
}

void icp_free(void *p) { std::free(p); }

const char *icp_strerror(int code)
{
    switch (code) {
    case ICP_OK: return "ok";
    case ICP_E_ARG: return "invalid argument";
    case ICP_E_HIP: return "HIP runtime error";
    case ICP_E_SIZE_MISMATCH: return "Point sets need to have the same number of points.";
    case ICP_E_TOO_FEW_POINTS: return "Need at least 4 point pairs";
    case ICP_E_NO_MODEL: return "model or scene not set";
    case ICP_E_RCCL: return "RCCL error";
    case ICP_E_NO_DEVICE: return "no HIP device";
    case ICP_E_IO: return "file could not be opened";
    case ICP_E_RANGE: return "coordinates outside the supported range";
    default: return "unknown error";
    }
}

} // extern "C"
