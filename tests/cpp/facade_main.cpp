// Closed-loop use of the C++ KiteNMPF facade the way nmpf_node.cpp drives the
// reference controller (set up, closest point, computeControl, read column N
// of getOptimalControl).  Prints one JSON line per step.
// Usage: facade_main <params.yaml> <steps> x0[0..14]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kite_nmpc/KiteNMPF.hpp"

int main(int argc, char** argv) {
    if (argc != 3 + 15) {
        std::fprintf(stderr, "usage: %s params.yaml steps x0(15)\n", argv[0]);
        return 2;
    }
    try {
        const kite_params p = kite_amd::LoadProperties(argv[1]);
        kite_amd::KiteNMPF nmpf(p);
        nmpf.createNLP();
        std::vector<double> x0(15);
        for (int i = 0; i < 15; ++i) x0[i] = std::atof(argv[3 + i]);
        x0[13] = nmpf.findClosestPointOnPath({x0[6], x0[7], x0[8]});
        const int steps = std::atoi(argv[2]);
        for (int s = 0; s < steps; ++s) {
            nmpf.computeControl(x0);
            const std::vector<double> U = nmpf.getOptimalControl();      // 4 x N, last column = u(t0)
            const std::vector<double> X = nmpf.getOptimalTrajetory();    // 15 x (N+1), last column = x(t0)
            const int N = (int)U.size() / 4;
            std::printf("{\"step\": %d, \"theta0\": %.17g, \"u0\": [%.17g, %.17g, %.17g, %.17g], "
                        "\"x1\": [", s, x0[13], U[(N - 1) * 4 + 0], U[(N - 1) * 4 + 1], U[(N - 1) * 4 + 2],
                        U[(N - 1) * 4 + 3]);
            for (int i = 0; i < 15; ++i) std::printf("%.17g%s", X[(size_t)(N - 1) * 15 + i], i < 14 ? ", " : "");
            std::printf("], \"status\": \"%s\", \"pos_error\": %.17g, \"vel_error\": %.17g, \"virt_state\": %.17g}\n",
                        nmpf.getStats().c_str(), nmpf.getPathError(), nmpf.getVelocityError(), nmpf.getVirtState());
            for (int i = 0; i < 15; ++i) x0[i] = X[(size_t)(N - 1) * 15 + i];   // closed loop on x(t0 + dt)
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
