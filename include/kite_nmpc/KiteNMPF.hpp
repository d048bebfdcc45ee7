// KiteNMPF.hpp -- header-only C++ facade over the C ABI (kite_nmpc.h) with the
// method names and semantics of the reference controller class
// (src/kite_control/kiteNMPF.h:10-118) for ONE kite, so that the ROS node
// (src/kite_control/nmpf_node.cpp) can switch with a one-line type change;
// see INTEGRATION.md.  casadi::DM arguments become std::vector<double>
// (matrices column-major, as DM stores them).
//
// Differences kept deliberately visible:
//   * the OCP is fixed at createNLP() (an RTI context), setters before it
//     configure, bound setters after it update the live context;
//   * getOptimalControl()/getOptimalTrajetory() keep the reference's shapes
//     (4 x (N+1), 15 x (N+1)) and REVERSED time order (last column = t0,
//     nmpf_node.cpp:124 reads column N).  The RTI has N piecewise-constant
//     controls (interval k starts at node k); column 0 (t = tf, where no
//     interval starts) repeats u_{N-1}, the control held up to tf;
//   * getStats() returns a string map (kite_amd::Dict) holding the IPOPT-style
//     "return_status" the node reads (nmpf_node.cpp:222-223), plus the RTI's
//     status bits;
//   * getPathFunction() returns a callable theta -> {x, y, z} instead of a
//     casadi::Function (nmpf_node.cpp:177-179 evaluates it per node);
//   * initialized() mirrors the reference, which never sets it (kiteNMPF.cpp:46).
#pragma once

#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "kite_nmpc.h"

// Facade version (compile-time): 2 = getStats() returns kite_amd::Dict (a
// string map with "return_status"; version 1 returned the status string),
// getOptimalControl() is 4 x (N+1) as the reference's (version 1: 4 x N),
// getPathFunction() and the C ABI's kite_nmpc_path_eval exist; 3 = arbitrary
// closed paths (FourierPath, the KiteNMPF(params, path) constructor, setPath).
#define KITE_NMPF_FACADE_VERSION 3

namespace kite_amd {

class KiteNmpcError : public std::runtime_error {
public:
    explicit KiteNmpcError(int code, const std::string& what)
        : std::runtime_error(what + ": " + kite_nmpc_strerror(code)), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void kite_check(int rc, const char* what) {
    if (rc < 0) throw KiteNmpcError(rc, what);
}

// casadi::Dict stand-in for getStats(): stats["return_status"] reads as in
// nmpf_node.cpp:222-223
using Dict = std::map<std::string, std::string>;

// KiteDynamics stand-in: the parameter set (kite_utils::LoadProperties, kite.cpp:7-76)
inline kite_params LoadProperties(const std::string& yaml_path) {
    kite_params p;
    kite_check(kite_params_load_yaml(yaml_path.c_str(), &p), "LoadProperties");
    return p;
}

// The path argument of KiteNMPF(kite, path) (kiteNMPF.h:14), which takes any
// casadi::Function theta -> R^3: a closed curve as a truncated Fourier series
// per axis, rotated by q as the node rotates its circle (nmpf_node.cpp:30-40).
// coef is 3 x (2K+1) row-major: axis a = x, y, z holds [c0, a1, b1, ..., aK, bK]
// of p_a(theta) = c0 + sum_k a_k cos(k theta) + b_k sin(k theta), K <= 8.
struct FourierPath {
    int harmonics = 0;
    std::vector<double> coef;
    double q[4] = {1.0, 0.0, 0.0, 0.0};
};

class KiteNMPF {
public:
    // KiteNMPF(shared_ptr<KiteDynamics>, path) (kiteNMPF.h:14): the dynamics are the
    // parameter set, the path is the rotated circle of the config (nmpf_node.cpp:30-40)
    explicit KiteNMPF(const kite_params& params, int N = 20, double dt = 0.05) : params_(params) {
        kite_nmpc_default_config(&cfg_);
        cfg_.N = N;
        cfg_.dt = dt;
    }
    // ... or any closed path
    KiteNMPF(const kite_params& params, const FourierPath& path, int N = 20, double dt = 0.05)
        : KiteNMPF(params, N, dt) {
        setPath(path);
    }
    // the reference declares setPath(SX) without defining it (kiteNMPF.h:36); here it
    // sets the tracked path: a live context is rebuilt (the path is part of the
    // OCP), so computeControl and getPathFunction always agree on it
    void setPath(const FourierPath& path) {
        const int K = path.harmonics;
        if (K < 1 || K > KITE_PATH_MAX_HARMONICS || path.coef.size() != (size_t)3 * (2 * K + 1))
            throw std::invalid_argument("setPath: coef must hold 3 x (2K+1) values, 1 <= K <= 8");
        std::memset(cfg_.path_fourier, 0, sizeof(cfg_.path_fourier));
        for (int a = 0; a < 3; ++a)
            for (int j = 0; j < 2 * K + 1; ++j) cfg_.path_fourier[a][j] = path.coef[(size_t)a * (2 * K + 1) + j];
        cfg_.path_harmonics = K;
        for (int i = 0; i < 4; ++i) cfg_.path_q[i] = path.q[i];
        if (ctx_) createNLP();
    }
    KiteNMPF(const kite_params& params, const kite_nmpc_config& cfg) : params_(params), cfg_(cfg) {}
    ~KiteNMPF() { kite_nmpc_destroy(ctx_); }
    KiteNMPF(const KiteNMPF&) = delete;
    KiteNMPF& operator=(const KiteNMPF&) = delete;

    // ---- setters (kiteNMPF.h:20-34) ----------------------------------------
    void setLBX(const std::vector<double>& v) { set_bounds(cfg_.lbx, v, 15, "setLBX"); }
    void setUBX(const std::vector<double>& v) { set_bounds(cfg_.ubx, v, 15, "setUBX"); }
    void setLBU(const std::vector<double>& v) { set_bounds(cfg_.lbu, v, 4, "setLBU"); }
    void setUBU(const std::vector<double>& v) { set_bounds(cfg_.ubu, v, 4, "setUBU"); }
    void setLBG(const std::vector<double>&) {}   // collocation equality bounds: no RTI counterpart
    void setUBG(const std::vector<double>&) {}
    // 15x15 / 4x4 diagonal scaling matrices (column-major) or their diagonals
    void setStateScaling(const std::vector<double>& S) { set_diag(cfg_.Sx, S, 15, "setStateScaling"); }
    void setControlScaling(const std::vector<double>& S) { set_diag(cfg_.Su, S, 4, "setControlScaling"); }
    // physical path speed (the reference stores Sx(14,14) * v, so it had to follow
    // setStateScaling; stored physical here, order-independent)
    void setReferenceVelocity(double v) {
        cfg_.vref = v;
        if (ctx_) kite_check(kite_nmpc_set_reference_velocity(ctx_, v), "setReferenceVelocity");
    }

    // constant world-frame wind of the prediction model, m/s (build extension,
    // kite_nmpc_set_wind: the reference model has no wind, kite.cpp:196); kept
    // across createNLP
    void setWind(double wx, double wy, double wz) {
        wind_[0] = wx; wind_[1] = wy; wind_[2] = wz;
        if (ctx_) kite_check(kite_nmpc_set_wind(ctx_, wind_), "setWind");
    }

    // ---- lifecycle (kiteNMPF.h:37-41) ---------------------------------------
    void createNLP() {
        kite_nmpc_destroy(ctx_);
        ctx_ = nullptr;
        kite_check(kite_nmpc_create(&params_, &cfg_, 1, &ctx_), "createNLP");
        kite_check(kite_nmpc_set_wind(ctx_, wind_), "createNLP");
        warm_ = false;
    }
    void enableWarmStart() { warm_ = true; }
    void disableWarmStart() {
        warm_ = false;
        if (ctx_) kite_check(kite_nmpc_reset(ctx_), "disableWarmStart");
    }
    // one RTI step from the physical 15-state X0 (kiteNMPF.cpp:199-316)
    void computeControl(const std::vector<double>& X0) {
        if (X0.size() != 15) throw std::invalid_argument("computeControl: X0 must have 15 entries");
        if (!ctx_) createNLP();
        if (!warm_) kite_check(kite_nmpc_reset(ctx_), "computeControl");
        const int N = cfg_.N;
        traj_.assign((size_t)(N + 1) * 15, 0.0);
        ctrl_.assign((size_t)N * 4, 0.0);
        kite_check(kite_nmpc_step(ctx_, X0.data(), u0_, traj_.data(), ctrl_.data(), &diag_, &status_),
                   "computeControl");
        warm_ = true;
    }

    // ---- getters (kiteNMPF.h:42-60) -----------------------------------------
    // 4 x (N+1), column-major, reference shape and column order: column N - k
    // = u_k, so the last column is u(t0); column 0 (t = tf) repeats u_{N-1}
    std::vector<double> getOptimalControl() const {
        const int N = cfg_.N;
        std::vector<double> out((size_t)4 * (N + 1));
        for (int k = 0; k <= N; ++k) {
            const int src = k < N ? k : N - 1;
            for (int c = 0; c < 4; ++c) out[(size_t)(N - k) * 4 + c] = ctrl_.empty() ? 0.0 : ctrl_[src * 4 + c];
        }
        return out;
    }
    // 15 x (N+1), column-major, reference column order: last column = x(t0)
    std::vector<double> getOptimalTrajetory() const {   // [sic] kiteNMPF.h:44
        const int N = cfg_.N;
        std::vector<double> out((size_t)15 * (N + 1));
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 15; ++i) out[(size_t)(N - k) * 15 + i] = traj_.empty() ? 0.0 : traj_[k * 15 + i];
        return out;
    }
    // getStats() (kiteNMPF.h:48): "return_status" as IPOPT names it
    // (kiteNMPF.cpp:303-313 checks these strings) + the RTI status bits
    Dict getStats() const {
        const char* rs = "Solve_Succeeded";
        if (status_ & KITE_ST_NAN) rs = "Invalid_Number_Detected";
        else if (status_ & KITE_ST_STEP_REJECTED) rs = "Restoration_Failed";
        else if (status_ & KITE_ST_QP_NOT_CONV) rs = "Maximum_Iterations_Exceeded";
        return Dict{{"return_status", rs}, {"status_bits", std::to_string(status_)}};
    }
    // getPathFunction() (kiteNMPF.h:46): P(theta) of the configured path
    // (the rotated circle of nmpf_node.cpp:30-40 or the FourierPath), evaluated on the host
    std::function<std::vector<double>(double)> getPathFunction() const {
        const kite_nmpc_config cfg = cfg_;
        return [cfg](double theta) {
            std::vector<double> P(3);
            kite_check(kite_nmpc_path_eval(&cfg, 1, &theta, P.data(), nullptr), "getPathFunction");
            return P;
        };
    }
    int32_t statusBits() const { return status_; }
    double getPathError() const { return diag_.pos_error; }
    double getVelocityError() const { return diag_.vel_error; }
    double getVirtState() const { return diag_.virt_state; }
    const kite_mpc_diagnostic& diagnostic() const { return diag_; }
    // u(t0) = [T, dE, dR, Uv] (what nmpf_node.cpp:120-138 publishes)
    const double* controlAtT0() const { return u0_; }
    bool initialized() const { return false; }   // never set in the reference (kiteNMPF.cpp:46)
    // findClosestPointOnPath (kiteNMPF.cpp:358-391)
    double findClosestPointOnPath(const std::vector<double>& position, double init_guess = 0.0) {
        if (position.size() != 3) throw std::invalid_argument("findClosestPointOnPath: 3 entries");
        if (!ctx_) createNLP();
        double th = 0.0;
        kite_check(kite_nmpc_closest_point(ctx_, 1, position.data(), &init_guess, &th), "findClosestPointOnPath");
        return th;
    }
    kite_nmpc_ctx* context() { return ctx_; }

private:
    void set_bounds(double* dst, const std::vector<double>& v, size_t n, const char* what) {
        if (v.size() != n) throw std::invalid_argument(std::string(what) + ": wrong size");
        std::memcpy(dst, v.data(), n * sizeof(double));
        if (ctx_) kite_check(kite_nmpc_set_bounds(ctx_, cfg_.lbx, cfg_.ubx, cfg_.lbu, cfg_.ubu), what);
    }
    void set_diag(double* dst, const std::vector<double>& S, size_t n, const char* what) {
        if (S.size() == n * n) {
            for (size_t i = 0; i < n; ++i) dst[i] = S[i * n + i];
        } else if (S.size() == n) {
            std::memcpy(dst, S.data(), n * sizeof(double));
        } else {
            throw std::invalid_argument(std::string(what) + ": wrong size");
        }
        if (ctx_) createNLP();   // scaling is part of the OCP: rebuild (reference: before createNLP)
    }

    kite_params params_;
    kite_nmpc_config cfg_;
    kite_nmpc_ctx* ctx_ = nullptr;
    bool warm_ = false;
    double wind_[3] = {0.0, 0.0, 0.0};
    std::vector<double> traj_, ctrl_;
    double u0_[4] = {0, 0, 0, 0};
    kite_mpc_diagnostic diag_{};
    int32_t status_ = 0;
};

}  // namespace kite_amd
