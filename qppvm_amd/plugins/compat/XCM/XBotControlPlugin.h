// XBotControlPlugin.h -- minimal compat subset of XCM / XBotInterface (ADVR) so that the
// plugin shells compile and run in this image (XCM, XBotInterface and Eigen are absent).
// Only the API the reference plugins call is reproduced:
//   XBot::XBotControlPlugin {init_control_plugin, on_start, on_stop, control_loop, close}
//   XBot::Handle::getRobotInterface / getPathToConfigFile
//   XBot::RobotInterface: getJointNum, get/setStiffness, get/setDamping, getDofIndex,
//                         getMotorPosition/Velocity, setReferenceFrom, move
//   XBot::ModelInterface: getJointNum, update, computeNonlinearTerm, getEffortLimits,
//                         getRobotState, set/getJointPosition, set/getJointVelocity,
//                         setJointEffort, getPose, getJacobian, getInertiaMatrix,
//                         computeJdotQdot, getPointPosition
//   REGISTER_XBOT_PLUGIN(name, class) -> extern "C" factory symbols
// Building against the real XCM is an install-time swap of this include directory; the
// linear-algebra types below stand in for Eigen's (column-major MatrixXd, fp64).
#pragma once

#include <cstddef>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace Eigen {

class VectorXd {
public:
    VectorXd() = default;
    explicit VectorXd(std::size_t n, double v = 0.0) : d_(n, v) {}
    std::size_t size() const { return d_.size(); }
    void resize(std::size_t n) { d_.resize(n); }
    VectorXd &setZero(std::size_t n) { d_.assign(n, 0.0); return *this; }
    VectorXd &setConstant(std::size_t n, double v) { d_.assign(n, v); return *this; }
    double &operator[](std::size_t i) { return d_[i]; }
    double operator[](std::size_t i) const { return d_[i]; }
    double &operator()(std::size_t i) { return d_[i]; }
    double operator()(std::size_t i) const { return d_[i]; }
    double *data() { return d_.data(); }
    const double *data() const { return d_.data(); }

private:
    std::vector<double> d_;
};

// dense matrix; column-major storage like Eigen's default MatrixXd (XBOT_COMPAT_ROW_MAJOR
// switches to row-major: the plugin shells read elements by (row, col), never through data(),
// so their results do not depend on the storage order -- tests/test_plugin.py checks both)
class MatrixXd {
public:
    MatrixXd() = default;
    MatrixXd(std::size_t r, std::size_t c) : r_(r), c_(c), d_(r * c, 0.0) {}
    std::size_t rows() const { return r_; }
    std::size_t cols() const { return c_; }
    void resize(std::size_t r, std::size_t c) { r_ = r; c_ = c; d_.assign(r * c, 0.0); }
#ifdef XBOT_COMPAT_ROW_MAJOR
    double &operator()(std::size_t i, std::size_t j) { return d_[i * c_ + j]; }
    double operator()(std::size_t i, std::size_t j) const { return d_[i * c_ + j]; }
#else
    double &operator()(std::size_t i, std::size_t j) { return d_[j * r_ + i]; }
    double operator()(std::size_t i, std::size_t j) const { return d_[j * r_ + i]; }
#endif
    double *data() { return d_.data(); }
    const double *data() const { return d_.data(); }

private:
    std::size_t r_ = 0, c_ = 0;
    std::vector<double> d_;
};

// [R | p] as 3x4 row-major (the top three rows of Affine3d::matrix())
struct Affine3d {
    double m[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
};

}  // namespace Eigen

namespace XBot {

namespace Sync {
enum Flag { Position = 1, Velocity = 2, Effort = 4, Impedance = 8 };
}

class ModelInterface;

class RobotInterface {
public:
    using Ptr = std::shared_ptr<RobotInterface>;
    virtual ~RobotInterface() = default;
    virtual int getJointNum() const = 0;
    virtual int getDofIndex(const std::string &joint) const = 0;
    virtual bool getStiffness(Eigen::VectorXd &k) const = 0;
    virtual bool getDamping(Eigen::VectorXd &d) const = 0;
    virtual bool setStiffness(const Eigen::VectorXd &k) = 0;
    virtual bool setDamping(const Eigen::VectorXd &d) = 0;
    virtual bool getMotorPosition(Eigen::VectorXd &q) const = 0;
    virtual bool getMotorVelocity(Eigen::VectorXd &qd) const = 0;
    virtual bool setReferenceFrom(const ModelInterface &model, Sync::Flag flag) = 0;
    // XBotInterface takes several Sync flags at once (ForceAcc.cpp:242: Position, Effort)
    bool setReferenceFrom(const ModelInterface &model, Sync::Flag a, Sync::Flag b)
    {
        return setReferenceFrom(model, static_cast<Sync::Flag>(a | b));
    }
    virtual bool move() = 0;
};

class ModelInterface {
public:
    using Ptr = std::shared_ptr<ModelInterface>;
    virtual ~ModelInterface() = default;
    virtual int getJointNum() const = 0;
    virtual bool update() = 0;
    virtual bool computeNonlinearTerm(Eigen::VectorXd &h) const = 0;
    virtual bool getEffortLimits(Eigen::VectorXd &tau_max) const = 0;
    virtual bool getRobotState(const std::string &name, Eigen::VectorXd &q) const = 0;
    virtual bool setJointPosition(const Eigen::VectorXd &q) = 0;
    virtual bool setJointVelocity(const Eigen::VectorXd &qd) = 0;
    virtual bool getJointPosition(Eigen::VectorXd &q) const = 0;
    virtual bool getJointVelocity(Eigen::VectorXd &qd) const = 0;
    virtual bool setJointEffort(const Eigen::VectorXd &tau) = 0;
    virtual bool getJointEffort(Eigen::VectorXd &tau) const = 0;
    virtual bool getPose(const std::string &link, Eigen::Affine3d &w_T_link) const = 0;
    virtual bool getJacobian(const std::string &link, Eigen::MatrixXd &J) const = 0;
    virtual bool getInertiaMatrix(Eigen::MatrixXd &M) const = 0;
    // used by the ForceAcc plugin (XBotInterface: computeJdotQdot(link, point, jdotqdot) and
    // getPointPosition(link, point, p), here at the link origin)
    virtual bool computeJdotQdot(const std::string &link, Eigen::VectorXd &jdqd) const
    {
        (void)link;
        jdqd.setZero(6);
        return true;
    }
    virtual bool getPointPosition(const std::string &link, Eigen::VectorXd &p) const
    {
        Eigen::Affine3d T;
        if (!getPose(link, T)) return false;
        p.setZero(3);
        for (int k = 0; k < 3; ++k) p[k] = T.m[4 * k + 3];
        return true;
    }
};

class Handle {
public:
    using Ptr = std::shared_ptr<Handle>;
    virtual ~Handle() = default;
    virtual RobotInterface::Ptr getRobotInterface() = 0;
    virtual ModelInterface::Ptr getModel() = 0; // compat: the model the plugin should use
    virtual std::string getPathToConfigFile() const = 0;
};

class XBotControlPlugin {
public:
    virtual ~XBotControlPlugin() = default;
    virtual bool init_control_plugin(Handle::Ptr handle) = 0;
    virtual void on_start(double time) {}
    virtual void on_stop(double time) {}
    virtual bool close() = 0;
    // the XBotCore RT thread calls this once per period
    void run(double time, double period) { control_loop(time, period); }

protected:
    virtual void control_loop(double time, double period) = 0;
};

}  // namespace XBot

// Factory symbols XBotCore dlopens [upstream loader contract, compat form].
#define REGISTER_XBOT_PLUGIN(plugin_name, scoped_class)                                   \
    extern "C" XBot::XBotControlPlugin *create_instance_##plugin_name() { return new scoped_class(); } \
    extern "C" void destroy_instance_##plugin_name(XBot::XBotControlPlugin *p) { delete p; }
