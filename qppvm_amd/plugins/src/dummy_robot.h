// dummy_robot.h -- XBotCore "dummy mode" stand-in for config 0 (BASELINE.json configs[0]):
// a synthetic CENTAURO-like model (n = 39 by default; the real URDF/YAML are not in the
// container) whose M(q), J(q), poses and h(q, qd) are smooth functions of the state, and a
// robot that integrates the commanded effort (semi-implicit Euler, the integration the
// reference leaves commented out at ForceAcc.cpp:225-226). Test/driver infrastructure only.
#pragma once

#include <XCM/XBotControlPlugin.h>

#include <cmath>
#include <random>
#include <string>
#include <vector>

namespace dummy {

struct Params {
    int n = 39;
    unsigned seed = 7;
    // links with a Jacobian / pose: QPPVM's end effectors (default), or a floating-base
    // quadruped (pelvis + 4 feet) for the ForceAcc plugin
    std::vector<std::string> links{"arm2_7", "arm1_7"};
    bool floating_base = false; // first 6 coordinates = floating base; gravity on its z row
    // Jacobian entry scale (lever arms, m). 0.2 keeps the operational-space inverse inertia
    // J M^-1 J^T ~ O(1) as on a real arm, so the reference gains (Dc = 70) are stable under the
    // 1 kHz explicit step (Dc * lambda_max(J M^-1 J^T) * dt < 2) and the 150 Nm limits bind only
    // now and then. 0.5 (--stress, the round-1 plant) gives lambda_max ~ 1e2: the closed loop
    // chatters, every joint saturates and the torques swap sides every tick -- a level-0
    // repair on every tick, kept as the worst case of the repair path.
    double jscale = 0.2;
};

inline Params quadruped(int n = 30)
{
    Params p;
    p.n = n;
    p.seed = 11;
    p.links = {"pelvis", "foot_fl", "foot_fr", "foot_hr", "foot_hl"};
    p.floating_base = true;
    p.jscale = 0.5;
    return p;
}

class Model : public XBot::ModelInterface {
public:
    explicit Model(const Params &p)
        : n_(p.n), links_(p.links), fb_(p.floating_base), q_(p.n, 0.0), qd_(p.n, 0.0), tau_(p.n, 0.0)
    {
        std::mt19937_64 g(p.seed);
        std::normal_distribution<double> N(0.0, 1.0);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        // fixed orthogonal basis (Gram-Schmidt of a random matrix) and base spectrum
        Q_.assign((size_t)n_ * n_, 0.0);
        for (auto &v : Q_) v = N(g);
        for (int c = 0; c < n_; ++c) {
            for (int k = 0; k < c; ++k) {
                double d = 0.0;
                for (int r = 0; r < n_; ++r) d += Q_[r * n_ + c] * Q_[r * n_ + k];
                for (int r = 0; r < n_; ++r) Q_[r * n_ + c] -= d * Q_[r * n_ + k];
            }
            double s = 0.0;
            for (int r = 0; r < n_; ++r) s += Q_[r * n_ + c] * Q_[r * n_ + c];
            s = 1.0 / std::sqrt(s);
            for (int r = 0; r < n_; ++r) Q_[r * n_ + c] *= s;
        }
        lam_.resize(n_);
        for (auto &l : lam_) l = std::exp(std::log(0.1) + U(g) * std::log(100.0)); // cond ~ 1e2
        const int nl = (int)links_.size();
        J0_.assign(nl, std::vector<double>((size_t)6 * n_, 0.0));
        p0_.assign(nl, std::vector<double>(3, 0.0));
        for (int t = 0; t < nl; ++t) {
            for (auto &v : J0_[t]) v = p.jscale * N(g);
            if (fb_ && t == 0) { // the base link moves with the floating base only
                for (auto &v : J0_[t]) v = 0.0;
                for (int r = 0; r < 6; ++r) J0_[t][r * n_ + r] = 1.0;
                for (int r = 0; r < 3; ++r)
                    for (int c = 3; c < 6; ++c) J0_[t][r * n_ + c] = 0.2 * N(g);
            }
            for (int k = 0; k < 3; ++k)
                p0_[t][k] = fb_ ? (t == 0 ? (k == 2 ? 0.6 : 0.0) : 0.4 * (k == 0 ? ((t & 1) ? 1 : -1) : (k == 1 ? (t < 3 ? 1 : -1) : 0)))
                                : (t == 0 ? -0.4 : 0.4) * (k == 1) + 0.5 * (k == 2);
        }
        psi_.resize(n_);
        for (auto &v : psi_) v = 6.28 * U(g);
    }
    int getJointNum() const override { return n_; }
    bool update() override { return true; }
    bool computeNonlinearTerm(Eigen::VectorXd &h) const override
    {
        h.setZero(n_);
        for (int j = 0; j < n_; ++j) h[j] = 10.0 * std::sin(q_[j] + psi_[j]) + 0.5 * qd_[j];
        if (fb_) h[2] += 50.0; // gravity on the base z row: the feet must push up
        return true;
    }
    bool getEffortLimits(Eigen::VectorXd &tmax) const override { tmax.setConstant(n_, 150.0); return true; }
    bool getJointLimits(Eigen::VectorXd &qmin, Eigen::VectorXd &qmax) const override
    {
        qmin.setConstant(n_, -0.3); // the dummy plant starts at q = 0 and moves by a few 0.1 rad
        qmax.setConstant(n_, 0.3);
        return true;
    }
    bool getRobotState(const std::string &, Eigen::VectorXd &q) const override { q.setZero(n_); return true; }
    bool setJointPosition(const Eigen::VectorXd &q) override { for (int j = 0; j < n_; ++j) q_[j] = q[j]; return true; }
    bool setJointVelocity(const Eigen::VectorXd &qd) override { for (int j = 0; j < n_; ++j) qd_[j] = qd[j]; return true; }
    bool getJointPosition(Eigen::VectorXd &q) const override { q.resize(n_); for (int j = 0; j < n_; ++j) q[j] = q_[j]; return true; }
    bool getJointVelocity(Eigen::VectorXd &qd) const override { qd.resize(n_); for (int j = 0; j < n_; ++j) qd[j] = qd_[j]; return true; }
    bool setJointEffort(const Eigen::VectorXd &tau) override { for (int j = 0; j < n_; ++j) tau_[j] = tau[j]; return true; }
    bool getJointEffort(Eigen::VectorXd &tau) const override { tau.resize(n_); for (int j = 0; j < n_; ++j) tau[j] = tau_[j]; return true; }
    bool getInertiaMatrix(Eigen::MatrixXd &M) const override
    {
        M.resize(n_, n_);
        std::vector<double> d(n_);
        for (int k = 0; k < n_; ++k) d[k] = lam_[k] * (1.0 + 0.2 * std::sin(q_[k]));
        for (int r = 0; r < n_; ++r)
            for (int c = r; c < n_; ++c) {
                double s = 0.0;
                for (int k = 0; k < n_; ++k) s += Q_[r * n_ + k] * d[k] * Q_[c * n_ + k];
                M(r, c) = s;
                M(c, r) = s;
            }
        return true;
    }
    bool getJacobian(const std::string &link, Eigen::MatrixXd &J) const override
    {
        const int t = task(link);
        J.resize(6, n_);
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < n_; ++c) J(r, c) = J0_[t][r * n_ + c] * (1.0 + 0.1 * std::cos(q_[c]));
        return true;
    }
    // d/dt (J) qd with J_rc = J0_rc (1 + 0.1 cos q_c): sum_c -0.1 J0_rc sin(q_c) qd_c^2
    bool computeJdotQdot(const std::string &link, const Eigen::Vector3d &, Eigen::Vector6d &jdqd) const override
    {
        const int t = task(link);
        jdqd.setZero();
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < n_; ++c) jdqd[r] -= 0.1 * J0_[t][r * n_ + c] * std::sin(q_[c]) * qd_[c] * qd_[c];
        return true;
    }
    bool getPose(const std::string &link, Eigen::Affine3d &T) const override
    {
        const int t = task(link);
        double w[3] = {0, 0, 0};
        for (int k = 0; k < 3; ++k) {
            double p = p0_[t][k], s = 0.0;
            for (int c = 0; c < n_; ++c) {
                p += 0.05 * J0_[t][k * n_ + c] * std::sin(q_[c]);
                s += 0.05 * J0_[t][(3 + k) * n_ + c] * std::sin(q_[c]);
            }
            T.translation()(k) = p;
            w[k] = s;
        }
        // rotation exp([w]x) (Rodrigues)
        const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        double K[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
        const double a = th > 1e-12 ? std::sin(th) / th : 1.0;
        const double b = th > 1e-12 ? (1 - std::cos(th)) / (th * th) : 0.5;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double kk = 0.0;
                for (int m = 0; m < 3; ++m) kk += K[r][m] * K[m][c];
                T.linear()(r, c) = (r == c ? 1.0 : 0.0) + a * K[r][c] + b * kk;
            }
        return true;
    }
    const std::vector<double> &effort() const { return tau_; }

private:
    int task(const std::string &link) const
    {
        for (size_t t = 0; t < links_.size(); ++t)
            if (links_[t] == link) return (int)t;
        return 0;
    }
    int n_;
    std::vector<std::string> links_;
    bool fb_;
    std::vector<double> q_, qd_, tau_, Q_, lam_, psi_;
    std::vector<std::vector<double>> J0_, p0_;
};

class Robot : public XBot::RobotInterface {
public:
    explicit Robot(int n)
        : n_(n), q_(Eigen::VectorXd::Zero(n)), qd_(Eigen::VectorXd::Zero(n)), k_(Eigen::VectorXd::Constant(n, 500.0)),
          d_(Eigen::VectorXd::Constant(n, 10.0))
    {
    }
    int getJointNum() const override { return n_; }
    int getDofIndex(const std::string &joint) const override
    {
        // CENTAURO-like naming: j_arm1_1..7 -> 0..6, j_arm2_1..7 -> 7..13
        if (joint.rfind("j_arm", 0) == 0 && joint.size() == 8) {
            const int arm = joint[5] - '1', j = joint[7] - '1';
            if (arm >= 0 && arm < 2 && j >= 0 && j < 7) return arm * 7 + j;
        }
        return -1;
    }
    bool getStiffness(Eigen::VectorXd &k) const override { k = k_; return true; }
    bool getDamping(Eigen::VectorXd &d) const override { d = d_; return true; }
    bool setStiffness(const Eigen::VectorXd &k) override { k_ = k; return true; }
    bool setDamping(const Eigen::VectorXd &d) override { d_ = d; return true; }
    bool getMotorPosition(Eigen::VectorXd &q) const override { q = q_; return true; }
    bool getMotorVelocity(Eigen::VectorXd &qd) const override { qd = qd_; return true; }
    using XBot::RobotInterface::setReferenceFrom;
    bool setReferenceFrom(const XBot::ModelInterface &model, XBot::Sync::Flag flag) override
    {
        if (flag & XBot::Sync::Effort) model.getJointEffort(tau_);
        if (flag & XBot::Sync::Position) model.getJointPosition(qref_);
        last_sync_ = flag;
        return true;
    }
    int last_sync() const { return last_sync_; }
    bool move() override { return true; }
    void set_state(const Eigen::VectorXd &q, const Eigen::VectorXd &qd) { q_ = q; qd_ = qd; }
    // dummy-mode kinematic step with a given acceleration (the integration the reference
    // leaves commented out at ForceAcc.cpp:225-226): semi-implicit Euler
    void step_qdd(const Eigen::VectorXd &qdd, double dt)
    {
        for (int j = 0; j < n_; ++j) {
            qd_[j] += dt * qdd[j];
            q_[j] += dt * qd_[j];
        }
    }
    // dummy-mode physics: q'' = M^-1 (tau - h), semi-implicit Euler
    void step(const Model &model, double dt)
    {
        if (tau_.size() != (Eigen::Index)n_) return;
        Eigen::MatrixXd M;
        Eigen::VectorXd h;
        model.getInertiaMatrix(M);
        model.computeNonlinearTerm(h);
        std::vector<double> L((size_t)n_ * n_), a(n_);
        for (int r = 0; r < n_; ++r)
            for (int c = 0; c < n_; ++c) L[(size_t)r * n_ + c] = M(r, c);
        for (int j = 0; j < n_; ++j) a[j] = tau_[j] - h[j];
        cholesky_solve(L, a);
        for (int j = 0; j < n_; ++j) {
            qd_[j] += dt * a[j];
            q_[j] += dt * qd_[j];
        }
    }

private:
    void cholesky_solve(std::vector<double> &A, std::vector<double> &b) const
    {
        const int n = n_;
        for (int j = 0; j < n; ++j) {
            double s = A[j * n + j];
            for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
            const double l = std::sqrt(s);
            A[j * n + j] = l;
            for (int i = j + 1; i < n; ++i) {
                double t = A[i * n + j];
                for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
                A[i * n + j] = t / l;
            }
        }
        for (int i = 0; i < n; ++i) {
            double t = b[i];
            for (int k = 0; k < i; ++k) t -= A[i * n + k] * b[k];
            b[i] = t / A[i * n + i];
        }
        for (int i = n - 1; i >= 0; --i) {
            double t = b[i];
            for (int k = i + 1; k < n; ++k) t -= A[k * n + i] * b[k];
            b[i] = t / A[i * n + i];
        }
    }
    int n_;
    Eigen::VectorXd q_, qd_, k_, d_, qref_;
    mutable Eigen::VectorXd tau_;
    int last_sync_ = 0;
};

class Handle : public XBot::Handle {
public:
    explicit Handle(const Params &p) : model_(std::make_shared<Model>(p)), robot_(std::make_shared<Robot>(p.n)) {}
    std::string getPathToConfigFile() const override { return "dummy://synthetic"; }
    XBot::RobotInterface::Ptr getRobotInterface() override { return robot_; }
    // the model XBot::ModelInterface::getModel(path) hands the plugin: the driver (the XBotCore
    // stand-in) registers it as the loader for this handle's config path
    std::shared_ptr<Model> model_ptr() { return model_; }
    void register_model()
    {
        auto m = model_;
        const std::string path = getPathToConfigFile();
        XBot::ModelInterface::setModelLoader([m, path](const std::string &p) {
            return p == path ? XBot::ModelInterface::Ptr(m) : XBot::ModelInterface::Ptr();
        });
    }
    Model &model() { return *model_; }
    Robot &robot() { return *robot_; }

private:
    std::shared_ptr<Model> model_;
    std::shared_ptr<Robot> robot_;
};

}  // namespace dummy
