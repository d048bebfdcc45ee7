// The reference ROS node's use of the controller (src/kite_control/nmpf_node.cpp),
// driven through the C++ KiteNMPF facade with every call the node makes:
//   ctor (nmpf_node.cpp:24-72): setControlScaling / setStateScaling (diagonal
//     matrices), setLBU / setUBU, setLBX / setUBX, setReferenceVelocity,
//     createNLP;
//   compute_control (:206-246): getOptimalTrajetory, first call
//     findClosestPointOnPath, later the delay-compensated state with theta,
//     thetadot from column N-2 and getStats()["return_status"], the vx clamp,
//     computeControl;
//   publish (:120-138): the last column of getOptimalControl;
//   publish_mpc_diagnostic (:191-204): getPathError, getVirtState,
//     getVelocityError;
//   publish_trajectory (:140-188): getOptimalTrajetory + getPathFunction per
//     column.
// The delay prediction (the node's CVODES ODESolver, :75-84, :218) is RK4 on
// the GPU here (kite_nmpc_predict, 0.1 s, 16 substeps); the plant is the plan's
// own prediction at t0 + dt.  Prints one JSON line per control step.
// Usage: facade_main <params.yaml> <steps> x0[0..12]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kite_nmpc/KiteNMPF.hpp"

static std::vector<double> diag_matrix(const std::vector<double>& d) {
    const size_t n = d.size();
    std::vector<double> m(n * n, 0.0);
    for (size_t i = 0; i < n; ++i) m[i * n + i] = d[i];
    return m;
}

int main(int argc, char** argv) {
    if (argc != 3 + 13) {
        std::fprintf(stderr, "usage: %s params.yaml steps x0(13)\n", argv[0]);
        return 2;
    }
    try {
        const kite_params p = kite_amd::LoadProperties(argv[1]);
        kite_amd::KiteNMPF controller(p);
        // ---- node constructor (nmpf_node.cpp:45-72) ----
        const double sat = 7.0 * M_PI / 180.0, inf = INFINITY, pi = M_PI;
        controller.setControlScaling(diag_matrix({1 / 0.15, 1 / 0.2618, 1 / 0.2618, 1 / 5.0}));
        controller.setStateScaling(diag_matrix({0.1, 1 / 3.0, 1 / 3.0, 1 / 2.0, 1 / 5.0, 1 / 2.0, 1 / 3.0, 1 / 3.0,
                                                1 / 3.0, 1.0, 1.0, 1.0, 1.0, 1 / 6.28, 1 / 6.28}));
        controller.setLBU({0.1, -sat, -sat, -5});
        controller.setUBU({0.15, sat, sat, 5});
        controller.setLBX({2.0, -inf, -inf, -4 * pi, -4 * pi, -4 * pi, -inf, -inf, -inf, -1.01, -1.01, -1.01, -1.01,
                           -inf, -inf});
        controller.setUBX({inf, inf, inf, 4 * pi, 4 * pi, 4 * pi, inf, inf, inf, 1.01, 1.01, 1.01, 1.01, inf, inf});
        controller.setReferenceVelocity(4.0);
        controller.createNLP();
        const double transport_delay = 0.1;

        std::vector<double> kite_state(13), control(3, 0.0);
        for (int i = 0; i < 13; ++i) kite_state[i] = std::atof(argv[3 + i]);
        const int steps = std::atoi(argv[2]);
        bool have_traj = false;
        for (int s = 0; s < steps; ++s) {
            // ---- compute_control (nmpf_node.cpp:206-246) ----
            std::vector<double> aug(15);
            std::string solve_status = "none";
            if (have_traj) {
                const std::vector<double> opt_traj = controller.getOptimalTrajetory();   // 15 x (N+1)
                const int cols = (int)opt_traj.size() / 15;
                // transport delay compensation (:218): RK4 prediction on the GPU
                std::vector<double> x15(15, 0.0), u4(4, 0.0), xp(15);
                for (int i = 0; i < 13; ++i) x15[i] = kite_state[i];
                for (int j = 0; j < 3; ++j) u4[j] = control[j];
                kite_amd::kite_check(kite_nmpc_predict(controller.context(), 1, x15.data(), u4.data(),
                                                       transport_delay, 16, xp.data()), "predict");
                for (int i = 0; i < 13; ++i) aug[i] = xp[i];
                aug[13] = opt_traj[(size_t)(cols - 3) * 15 + 13];                      // column size2 - 3 (:220)
                aug[14] = opt_traj[(size_t)(cols - 3) * 15 + 14];
                kite_amd::Dict stats = controller.getStats();                           // (:222-223)
                solve_status = static_cast<std::string>(stats["return_status"]);
            } else {
                const double closest_point =
                    controller.findClosestPointOnPath({kite_state[6], kite_state[7], kite_state[8]});
                for (int i = 0; i < 13; ++i) aug[i] = kite_state[i];
                aug[13] = closest_point;
                aug[14] = 0.0;
            }
            if (aug[0] < 2.1) aug[0] = 2.1;                                            // (:241-243)
            controller.computeControl(aug);
            have_traj = true;
            // ---- publish (:120-138) ----
            const std::vector<double> opt_ctl = controller.getOptimalControl();        // 4 x (N+1)
            const int ccols = (int)opt_ctl.size() / 4;
            for (int j = 0; j < 3; ++j) control[j] = opt_ctl[(size_t)(ccols - 1) * 4 + j];
            // ---- publish_trajectory (:140-188) ----
            const std::vector<double> T = controller.getOptimalTrajetory();
            const int cols = (int)T.size() / 15;
            auto path = controller.getPathFunction();
            const std::vector<double> virt_t0 = path(T[(size_t)(cols - 1) * 15 + 13]);
            const std::vector<double> virt_tf = path(T[13]);
            std::printf("{\"step\": %d, \"prev_status\": \"%s\", \"ctrl_cols\": %d, \"traj_cols\": %d, \"aug\": [",
                        s, solve_status.c_str(), ccols, cols);
            for (int i = 0; i < 15; ++i) std::printf("%.17g%s", aug[i], i < 14 ? ", " : "");
            std::printf("], \"control\": [%.17g, %.17g, %.17g], \"x1\": [", control[0], control[1], control[2]);
            for (int i = 0; i < 15; ++i) std::printf("%.17g%s", T[(size_t)(cols - 2) * 15 + i], i < 14 ? ", " : "");
            // ---- publish_mpc_diagnostic (:191-204) ----
            std::printf("], \"status\": \"%s\", \"pos_error\": %.17g, \"vel_error\": %.17g, \"virt_state\": %.17g, "
                        "\"virt_t0\": [%.17g, %.17g, %.17g], \"virt_tf\": [%.17g, %.17g, %.17g]}\n",
                        controller.getStats()["return_status"].c_str(), controller.getPathError(),
                        controller.getVelocityError(), controller.getVirtState(), virt_t0[0], virt_t0[1], virt_t0[2],
                        virt_tf[0], virt_tf[1], virt_tf[2]);
            // plant: the plan's state at t0 + dt (column N-1)
            for (int i = 0; i < 13; ++i) kite_state[i] = T[(size_t)(cols - 2) * 15 + i];
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
