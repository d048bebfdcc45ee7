// getPathFunction() of a KiteNMPF built with an arbitrary closed path (the
// KiteNMPF(kite, path) constructor, kiteNMPF.h:14) -- no GPU: the path
// evaluator is host arithmetic.  Prints theta x y z per line.
#include <cstdio>
#include <cstdlib>

#include "kite_nmpc/KiteNMPF.hpp"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    kite_amd::FourierPath path;
    path.harmonics = 3;
    path.coef.assign(3 * 7, 0.0);
    for (int i = 0; i < 21; ++i) path.coef[i] = std::atof(argv[1 + i]);
    path.q[0] = std::atof(argv[22]); path.q[1] = std::atof(argv[23]);
    path.q[2] = std::atof(argv[24]); path.q[3] = std::atof(argv[25]);
    const kite_params p = kite_amd::LoadProperties(argv[26]);
    kite_amd::KiteNMPF controller(p, path);
    auto P = controller.getPathFunction();
    for (int i = 0; i <= 8; ++i) {
        const double th = -3.0 + 0.75 * i;
        const std::vector<double> v = P(th);
        std::printf("%.17g %.17g %.17g %.17g\n", th, v[0], v[1], v[2]);
    }
    return 0;
}
