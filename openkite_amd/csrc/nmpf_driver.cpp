// nmpf_driver -- closed-loop fleet driver: the openKITE simulator node
// (src/kite_model/simulator.cpp, 50 Hz RK4 plant) and the NMPC node
// (src/kite_control/nmpf_node.cpp: closest-point initialisation, delay
// compensation, minimal-speed clamp, computeControl, mpc_diagnostic publish)
// for B kites at once, on the C ABI of libkite_nmpc.so.  Replaces the ROS
// plumbing; emits the mpc_diagnostic stream (msg/mpc_diagnostic.msg) as JSONL.
//
//   nmpf_driver [--params yaml] [--batch B] [--steps S] [--x0 file.csv]
//               [--ctrl-every K] [--sim-dt h] [--delay d] [--trace T] [--seed s]
//               [--out file.jsonl] [--device i]
//
// Timeline (per control step, all kites in lockstep):
//   measure x (13 plant states) -> kite_nmpc_step (prologue predicts over
//   `delay` when warm) -> u(t0) applied to the plant for K plant steps of
//   sim-dt (kite_nmpc_predict, RK4 with 4 substeps per plant step, the
//   simulator's integrator).  Per step one summary line; per traced kite one
//   mpc_diagnostic line.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "kite_nmpc/kite_nmpc.h"

namespace {

struct Args {
    std::string params = "data/umx_radian.yaml";
    std::string x0_file, out_file;
    int batch = 64, steps = 100, ctrl_every = 3, trace = 1, device = 0;
    double sim_dt = 0.02, delay = 0.1;
    unsigned long long seed = 20261015ull;
};

[[noreturn]] void usage(const char* argv0) {
    std::fprintf(stderr,
                 "usage: %s [--params yaml] [--batch B] [--steps S] [--x0 file.csv] [--ctrl-every K]\n"
                 "          [--sim-dt h] [--delay d] [--trace T] [--seed s] [--out file.jsonl] [--device i]\n",
                 argv0);
    std::exit(2);
}

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) usage(argv[0]);
            return argv[++i];
        };
        if (k == "--params") a.params = val();
        else if (k == "--batch") a.batch = std::atoi(val());
        else if (k == "--steps") a.steps = std::atoi(val());
        else if (k == "--x0") a.x0_file = val();
        else if (k == "--ctrl-every") a.ctrl_every = std::atoi(val());
        else if (k == "--sim-dt") a.sim_dt = std::atof(val());
        else if (k == "--delay") a.delay = std::atof(val());
        else if (k == "--trace") a.trace = std::atoi(val());
        else if (k == "--seed") a.seed = std::strtoull(val(), nullptr, 10);
        else if (k == "--out") a.out_file = val();
        else if (k == "--device") a.device = std::atoi(val());
        else usage(argv[0]);
    }
    if (a.batch < 1 || a.steps < 0 || a.ctrl_every < 1 || !(a.sim_dt > 0) || a.trace < 0) usage(argv[0]);
    return a;
}

// launch/simulator.launch:3 initial state, perturbed per kite (seeded)
void synthetic_states(int B, unsigned long long seed, std::vector<double>& x) {
    const double base[13] = {4.4, 0.44, 1.73, 0.81, -1.73, -1.53, -0.46, -2.68, 0.64,
                             -0.0289, 0.1587, 0.4304, 0.8881};
    x.assign((size_t)B * 13, 0.0);
    for (int b = 0; b < B; ++b) {
        std::mt19937_64 rng(seed + (unsigned long long)b);
        std::uniform_real_distribution<double> U(-1.0, 1.0);
        double* s = &x[(size_t)b * 13];
        for (int i = 0; i < 13; ++i) s[i] = base[i];
        for (int i = 0; i < 3; ++i) s[i] += 0.5 * U(rng);
        for (int i = 3; i < 6; ++i) s[i] += 0.3 * U(rng);
        for (int i = 6; i < 9; ++i) s[i] += 0.05 * U(rng);
        double n = 0;
        for (int i = 9; i < 13; ++i) { s[i] += 0.02 * U(rng); n += s[i] * s[i]; }
        n = std::sqrt(n);
        for (int i = 9; i < 13; ++i) s[i] /= n;
    }
}

bool read_csv(const std::string& path, int B, std::vector<double>& x) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    x.assign((size_t)B * 13, 0.0);
    for (size_t i = 0; i < x.size(); ++i) {
        if (std::fscanf(f, " %lf ,", &x[i]) != 1) { std::fclose(f); return false; }
    }
    std::fclose(f);
    return true;
}

int fail(const char* what, int rc) {
    std::fprintf(stderr, "nmpf_driver: %s: %s (%d)\n", what, kite_nmpc_strerror(rc), rc);
    return 1;
}

// %.17g that stays valid JSON (NaN / inf -> null)
void jnum(FILE* f, double v, const char* sep) {
    if (std::isfinite(v)) std::fprintf(f, "%.17g%s", v, sep);
    else std::fprintf(f, "null%s", sep);
}

}  // namespace

int main(int argc, char** argv) {
    const Args a = parse(argc, argv);
    const int B = a.batch;
    kite_params kp;
    int rc = kite_params_load_yaml(a.params.c_str(), &kp);
    if (rc) return fail("load params", rc);
    kite_nmpc_config cfg;
    kite_nmpc_default_config(&cfg);
    cfg.device = a.device;
    cfg.delay = a.delay;                  // node: 0.1 s (nmpf_node.cpp:74)
    kite_nmpc_ctx* ctx = nullptr;
    rc = kite_nmpc_create(&kp, &cfg, B, &ctx);
    if (rc) return fail("create", rc);

    std::vector<double> plant;            // B x 13 plant states
    if (!a.x0_file.empty()) {
        if (!read_csv(a.x0_file, B, plant)) { std::fprintf(stderr, "nmpf_driver: cannot read %s\n", a.x0_file.c_str()); return 1; }
    } else {
        synthetic_states(B, a.seed, plant);
    }
    FILE* out = a.out_file.empty() ? stdout : std::fopen(a.out_file.c_str(), "w");
    if (!out) { std::fprintf(stderr, "nmpf_driver: cannot open %s\n", a.out_file.c_str()); return 1; }

    const int N = cfg.N;
    std::vector<double> x0((size_t)B * 15), u0((size_t)B * 4), traj((size_t)B * (N + 1) * 15);
    std::vector<double> pos((size_t)B * 3), guess((size_t)B, 0.0), theta((size_t)B), x15((size_t)B * 15),
        u4((size_t)B * 4, 0.0), xn((size_t)B * 15);
    std::vector<kite_mpc_diagnostic> diag(B);
    std::vector<int32_t> status(B);

    // initialisation (nmpf_node.cpp:233-236): closest point, thetadot = 0
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < 3; ++i) pos[(size_t)b * 3 + i] = plant[(size_t)b * 13 + 6 + i];
    rc = kite_nmpc_closest_point(ctx, B, pos.data(), guess.data(), theta.data());
    if (rc) return fail("closest point", rc);

    double t = 0.0;
    for (int s = 0; s < a.steps; ++s) {
        // measurement: plant state; theta/thetadot only matter on the cold step
        // (warm steps take them from the previous plan, nmpf_node.cpp:220)
        for (int b = 0; b < B; ++b) {
            double* xb = &x0[(size_t)b * 15];
            std::memcpy(xb, &plant[(size_t)b * 13], 13 * sizeof(double));
            xb[13] = s == 0 ? theta[b] : traj[(size_t)b * (N + 1) * 15 + 15 + 13];
            xb[14] = s == 0 ? 0.0 : traj[(size_t)b * (N + 1) * 15 + 15 + 14];
        }
        const auto c0 = std::chrono::steady_clock::now();
        rc = kite_nmpc_step(ctx, x0.data(), u0.data(), traj.data(), nullptr, diag.data(), status.data());
        if (rc) return fail("step", rc);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();

        // publish: summary + traced kites' mpc_diagnostic records
        double pe_sum = 0, pe_max = 0, ve_sum = 0, th_sum = 0;
        int n_rej = 0, n_nan = 0, n_nc = 0, n_rst = 0;
        int n_fin = 0;
        for (int b = 0; b < B; ++b) {
            if (std::isfinite(diag[b].pos_error) && std::isfinite(diag[b].vel_error) && std::isfinite(diag[b].virt_state)) {
                pe_sum += diag[b].pos_error; pe_max = std::fmax(pe_max, diag[b].pos_error);
                ve_sum += diag[b].vel_error; th_sum += diag[b].virt_state;
                ++n_fin;
            }
            n_nan += (status[b] & KITE_ST_NAN) != 0;
            n_nc += (status[b] & KITE_ST_QP_NOT_CONV) != 0;
            n_rej += (status[b] & KITE_ST_STEP_REJECTED) != 0;
            n_rst += (status[b] & KITE_ST_RESTART) != 0;
        }
        // aggregates over the finite kites only (a NaN kite restarts next step)
        std::fprintf(out,
                     "{\"type\": \"step\", \"step\": %d, \"t\": %.4f, \"comp_time_ms\": %.4f, \"pos_error_mean\": %.9g, "
                     "\"pos_error_max\": %.9g, \"vel_error_mean\": %.9g, \"virt_state_mean\": %.9g, \"nan\": %d, "
                     "\"qp_not_converged\": %d, \"step_rejected\": %d, \"restarts\": %d}\n",
                     s, t, ms, pe_sum / std::max(1, n_fin), pe_max, ve_sum / std::max(1, n_fin),
                     th_sum / std::max(1, n_fin), n_nan, n_nc, n_rej, n_rst);
        for (int b = 0; b < std::min(a.trace, B); ++b) {
            const double* ub = &u0[(size_t)b * 4];
            std::fprintf(out, "{\"type\": \"mpc_diagnostic\", \"kite\": %d, \"step\": %d, \"pos_error\": ", b, s);
            jnum(out, diag[b].pos_error, ", \"vel_error\": ");
            jnum(out, diag[b].vel_error, ", \"cost\": ");
            jnum(out, diag[b].cost, ", \"virt_state\": ");
            jnum(out, diag[b].virt_state, ", \"virt_ctrl\": ");
            jnum(out, diag[b].virt_ctrl, "");
            std::fprintf(out, ", \"comp_time_ms\": %.4f, \"status\": %d, \"u\": [", ms, status[b]);
            for (int c = 0; c < 4; ++c) jnum(out, ub[c], c < 3 ? ", " : "], \"x\": [");
            for (int i = 0; i < 13; ++i) jnum(out, plant[(size_t)b * 13 + i], i < 12 ? ", " : "]}\n");
        }

        // plant: u(t0) held for ctrl_every simulator steps (simulator.cpp:43-51)
        for (int b = 0; b < B; ++b) {
            std::memcpy(&u4[(size_t)b * 4], &u0[(size_t)b * 4], 3 * sizeof(double));
            u4[(size_t)b * 4 + 3] = 0.0;
        }
        for (int k = 0; k < a.ctrl_every; ++k) {
            for (int b = 0; b < B; ++b) {
                std::memcpy(&x15[(size_t)b * 15], &plant[(size_t)b * 13], 13 * sizeof(double));
                x15[(size_t)b * 15 + 13] = 0.0;
                x15[(size_t)b * 15 + 14] = 0.0;
            }
            rc = kite_nmpc_predict(ctx, B, x15.data(), u4.data(), a.sim_dt, 4, xn.data());
            if (rc) return fail("plant", rc);
            for (int b = 0; b < B; ++b) std::memcpy(&plant[(size_t)b * 13], &xn[(size_t)b * 15], 13 * sizeof(double));
            t += a.sim_dt;
        }
    }
    if (out != stdout) std::fclose(out);
    kite_nmpc_destroy(ctx);
    return 0;
}
