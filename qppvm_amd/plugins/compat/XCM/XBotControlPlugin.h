// XBotControlPlugin.h -- compat subset of XCM / XBotInterface / Eigen / KDL (ADVR) so that the
// plugin shells compile and run in this image, where none of them is installed. It reproduces
// only the API the reference plugins call, with the reference's own
// spellings, so the shells contain nothing a real XCM + XBotInterface + Eigen + KDL build would
// reject:
//   Eigen   VectorXd (Zero, Constant, setZero, setConstant, arithmetic, the << comma initializer),
//           MatrixXd, Matrix3d,
//           Matrix4d, Vector3d (Zero, UnitZ), Vector6d (XBotInterface's typedef),
//           Affine3d (linear(), translation(), matrix())
//   KDL     Frame {M, p}, Vector (x()/y()/z() getters and setters: QPPVMPlugin.cpp:219-221)
//   XBot    XBotControlPlugin {init_control_plugin, on_start, on_stop, control_loop, close},
//           Handle::getRobotInterface / getPathToConfigFile, JointIdMap,
//           RobotInterface (getJointNum, get/setStiffness, get/setDamping, getDofIndex,
//           getMotorPosition/Velocity incl. the JointIdMap overloads, setReferenceFrom, move),
//           ModelInterface (static getModel(path), syncFrom, update, initLog, log,
//           computeNonlinearTerm, getEffortLimits, getRobotState, set/getJointPosition,
//           set/getJointVelocity incl. JointIdMap, setJointEffort, getPose (Affine3d and
//           KDL::Frame), getJacobian, getInertiaMatrix, computeJdotQdot, getPointPosition)
//   REGISTER_XBOT_PLUGIN(name, class) and REGISTER_XBOT_PLUGIN_(class) -> extern "C" factories
// Building against the real libraries is an install-time swap of this include directory.
//
// Two hooks exist only for the host runtime that stands in for XBotCore (the dummy-mode driver),
// never for the plugins: ModelInterface::setModelLoader (what getModel(path) returns; real
// XBotInterface loads the URDF/SRDF a YAML config names) and MatLogger's file format.
#pragma once

#include <cstddef>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace Eigen {

using Index = std::ptrdiff_t;

// comma initializer (v << a, b, c, ...): coefficients in row-major order, as Eigen fills them
template <class D>
struct CommaInitializer {
    D &m;
    Index k;
    CommaInitializer &operator,(double v)
    {
        m.comma_set(k++, v);
        return *this;
    }
};

// fixed-size dense matrix, column-major like Eigen::Matrix<double, R, C>
template <int R, int C>
class Matrix {
public:
    Matrix() { setZero(); }
    static Matrix Zero() { return Matrix(); }
    static Matrix Identity()
    {
        Matrix m;
        for (int k = 0; k < (R < C ? R : C); ++k) m(k, k) = 1.0;
        return m;
    }
    static Matrix Unit(Index i)
    {
        static_assert(C == 1, "a unit vector");
        Matrix m;
        m(i) = 1.0;
        return m;
    }
    static Matrix UnitX() { return Unit(0); }
    static Matrix UnitY() { return Unit(1); }
    static Matrix UnitZ() { return Unit(2); }
    static constexpr Index rows() { return R; }
    static constexpr Index cols() { return C; }
    static constexpr Index size() { return R * C; }
    Matrix &setZero()
    {
        for (double &v : d_) v = 0.0;
        return *this;
    }
    Matrix &setIdentity() { return *this = Identity(); }
    double &operator()(Index i, Index j) { return d_[j * R + i]; }
    double operator()(Index i, Index j) const { return d_[j * R + i]; }
    double &operator()(Index i) { return d_[i]; }
    double operator()(Index i) const { return d_[i]; }
    double &operator[](Index i) { return d_[i]; }
    double operator[](Index i) const { return d_[i]; }
    double x() const { return d_[0]; }
    double y() const { return d_[1]; }
    double z() const { return d_[2]; }
    double *data() { return d_; }
    const double *data() const { return d_; }
    Matrix operator+(const Matrix &o) const { return zip(o, 1.0); }
    Matrix operator-(const Matrix &o) const { return zip(o, -1.0); }
    Matrix operator-() const { return *this * -1.0; }
    Matrix operator*(double s) const
    {
        Matrix m;
        for (int k = 0; k < R * C; ++k) m.d_[k] = d_[k] * s;
        return m;
    }
    friend Matrix operator*(double s, const Matrix &m) { return m * s; }
    Matrix &operator+=(const Matrix &o) { return *this = *this + o; }
    Matrix &operator-=(const Matrix &o) { return *this = *this - o; }
    CommaInitializer<Matrix> operator<<(double v)
    {
        comma_set(0, v);
        return CommaInitializer<Matrix>{*this, 1};
    }
    void comma_set(Index k, double v) { (*this)(k / C, k % C) = v; }

private:
    Matrix zip(const Matrix &o, double s) const
    {
        Matrix m;
        for (int k = 0; k < R * C; ++k) m.d_[k] = d_[k] + s * o.d_[k];
        return m;
    }
    double d_[R * C];
};

using Matrix3d = Matrix<3, 3>;
using Matrix4d = Matrix<4, 4>;
using Vector3d = Matrix<3, 1>;
using Vector6d = Matrix<6, 1>; // XBotInterface adds this typedef to namespace Eigen

// dynamic vector. As in Eigen, VectorXd(n) takes a size and nothing else (Eigen rejects a
// (size, value) pair at compile time: FLOATING_POINT_ARGUMENT_PASSED__INTEGER_WAS_EXPECTED), so
// the shells fill vectors through Zero / Constant / setZero / setConstant
class VectorXd {
public:
    VectorXd() = default;
    explicit VectorXd(Index n) : d_((std::size_t)n, 0.0) {} // Eigen leaves the values uninitialised
    VectorXd(Index, double) = delete;
    template <int R>
    VectorXd(const Matrix<R, 1> &v) : d_(v.data(), v.data() + R) {}
    static VectorXd Zero(Index n) { return VectorXd(n); }
    static VectorXd Constant(Index n, double v) { return VectorXd(n).setConstant(v); }
    Index size() const { return (Index)d_.size(); }
    void resize(Index n) { d_.resize((std::size_t)n); }
    VectorXd &setZero() { return setConstant(0.0); }
    VectorXd &setZero(Index n) { return setConstant(n, 0.0); }
    VectorXd &setConstant(double v)
    {
        for (double &x : d_) x = v;
        return *this;
    }
    VectorXd &setConstant(Index n, double v)
    {
        d_.assign((std::size_t)n, v);
        return *this;
    }
    double &operator[](Index i) { return d_[(std::size_t)i]; }
    double operator[](Index i) const { return d_[(std::size_t)i]; }
    double &operator()(Index i) { return d_[(std::size_t)i]; }
    double operator()(Index i) const { return d_[(std::size_t)i]; }
    double *data() { return d_.data(); }
    const double *data() const { return d_.data(); }
    CommaInitializer<VectorXd> operator<<(double v)
    {
        comma_set(0, v);
        return CommaInitializer<VectorXd>{*this, 1};
    }
    void comma_set(Index k, double v) { d_.at((std::size_t)k) = v; }
    VectorXd operator+(const VectorXd &o) const { return zip(o, 1.0); }
    VectorXd operator-(const VectorXd &o) const { return zip(o, -1.0); }
    VectorXd operator-() const { return *this * -1.0; }
    VectorXd operator*(double s) const
    {
        VectorXd r(*this);
        return r *= s;
    }
    friend VectorXd operator*(double s, const VectorXd &v) { return v * s; }
    VectorXd &operator+=(const VectorXd &o)
    {
        for (std::size_t k = 0; k < d_.size(); ++k) d_[k] += o.d_[k];
        return *this;
    }
    VectorXd &operator-=(const VectorXd &o)
    {
        for (std::size_t k = 0; k < d_.size(); ++k) d_[k] -= o.d_[k];
        return *this;
    }
    VectorXd &operator*=(double s)
    {
        for (double &x : d_) x *= s;
        return *this;
    }
    VectorXd &operator/=(double s)
    {
        for (double &x : d_) x /= s;
        return *this;
    }

private:
    VectorXd zip(const VectorXd &o, double s) const
    {
        VectorXd r(*this);
        for (std::size_t k = 0; k < d_.size(); ++k) r.d_[k] += s * o.d_[k];
        return r;
    }
    std::vector<double> d_;
};

// dynamic matrix; column-major storage like Eigen's default MatrixXd (XBOT_COMPAT_ROW_MAJOR
// switches to row-major: the plugin shells read elements by (row, col), never through data(),
// so their results do not depend on the storage order -- tests/test_plugin.py checks both)
class MatrixXd {
public:
    MatrixXd() = default;
    MatrixXd(Index r, Index c) : r_(r), c_(c), d_((std::size_t)(r * c), 0.0) {}
    static MatrixXd Zero(Index r, Index c) { return MatrixXd(r, c); }
    static MatrixXd Identity(Index r, Index c) { return MatrixXd(r, c).setIdentity(r, c); }
    Index rows() const { return r_; }
    Index cols() const { return c_; }
    void resize(Index r, Index c)
    {
        r_ = r;
        c_ = c;
        d_.assign((std::size_t)(r * c), 0.0);
    }
    MatrixXd &setZero(Index r, Index c)
    {
        resize(r, c);
        return *this;
    }
    MatrixXd &setIdentity(Index r, Index c)
    {
        resize(r, c);
        for (Index k = 0; k < (r < c ? r : c); ++k) (*this)(k, k) = 1.0;
        return *this;
    }
#ifdef XBOT_COMPAT_ROW_MAJOR
    double &operator()(Index i, Index j) { return d_[(std::size_t)(i * c_ + j)]; }
    double operator()(Index i, Index j) const { return d_[(std::size_t)(i * c_ + j)]; }
#else
    double &operator()(Index i, Index j) { return d_[(std::size_t)(j * r_ + i)]; }
    double operator()(Index i, Index j) const { return d_[(std::size_t)(j * r_ + i)]; }
#endif
    double *data() { return d_.data(); }
    const double *data() const { return d_.data(); }

private:
    Index r_ = 0, c_ = 0;
    std::vector<double> d_;
};

// rigid transform (Eigen::Transform<double, 3, Affine>): linear block and translation
class Affine3d {
public:
    Affine3d() : L_(Matrix3d::Identity()) {} // Eigen leaves it uninitialised
    static Affine3d Identity() { return Affine3d(); }
    Affine3d &setIdentity() { return *this = Affine3d(); }
    Matrix3d &linear() { return L_; }
    const Matrix3d &linear() const { return L_; }
    Matrix3d rotation() const { return L_; } // a rigid transform's linear part
    Vector3d &translation() { return t_; }
    const Vector3d &translation() const { return t_; }
    Matrix4d matrix() const
    {
        Matrix4d m = Matrix4d::Identity();
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) m(r, c) = L_(r, c);
            m(r, 3) = t_(r);
        }
        return m;
    }
    Vector3d operator*(const Vector3d &p) const
    {
        Vector3d o = t_;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) o(r) += L_(r, c) * p(c);
        return o;
    }

private:
    Matrix3d L_;
    Vector3d t_;
};

}  // namespace Eigen

namespace KDL {

class Vector {
public:
    Vector() = default;
    Vector(double x, double y, double z) : data{x, y, z} {}
    double x() const { return data[0]; }
    double y() const { return data[1]; }
    double z() const { return data[2]; }
    void x(double v) { data[0] = v; }
    void y(double v) { data[1] = v; }
    void z(double v) { data[2] = v; }
    double operator()(int i) const { return data[i]; }
    double &operator()(int i) { return data[i]; }
    double data[3] = {0.0, 0.0, 0.0};
};

class Rotation { // row-major 3x3, as KDL stores it
public:
    double operator()(int i, int j) const { return data[3 * i + j]; }
    double &operator()(int i, int j) { return data[3 * i + j]; }
    static Rotation Identity() { return Rotation(); }
    double data[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
};

class Frame {
public:
    Rotation M;
    Vector p;
};

}  // namespace KDL

namespace XBot {

namespace Sync {
enum Flag { Position = 1, Velocity = 2, Effort = 4, Impedance = 8 };
}

// joint id -> value (XBotInterface's JointIdMap); compat joint ids are the joint indices
using JointIdMap = std::unordered_map<int, double>;

class MatLogger;
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
    bool getMotorPosition(JointIdMap &q) const { return to_map(&RobotInterface::getMotorPosition, q); }
    bool getMotorVelocity(JointIdMap &qd) const { return to_map(&RobotInterface::getMotorVelocity, qd); }
    virtual bool setReferenceFrom(const ModelInterface &model, Sync::Flag flag) = 0;
    // XBotInterface takes several Sync flags at once (ForceAcc.cpp:242: Position, Effort)
    bool setReferenceFrom(const ModelInterface &model, Sync::Flag a, Sync::Flag b)
    {
        return setReferenceFrom(model, static_cast<Sync::Flag>(a | b));
    }
    virtual bool move() = 0;

private:
    bool to_map(bool (RobotInterface::*get)(Eigen::VectorXd &) const, JointIdMap &m) const
    {
        if (!(this->*get)(map_buf_)) return false;
        for (Eigen::Index j = 0; j < map_buf_.size(); ++j) m[(int)j] = map_buf_[j];
        return true;
    }
    mutable Eigen::VectorXd map_buf_; // (reused: no allocation per call once sized)
};

class ModelInterface {
public:
    using Ptr = std::shared_ptr<ModelInterface>;
    using Loader = std::function<Ptr(const std::string &path_to_config_file)>;
    virtual ~ModelInterface() = default;

    // XBotInterface: the model a YAML config (URDF + SRDF) describes (QPPVMPlugin.cpp:50,
    // ForceAcc.cpp:43). Compat: whatever the host runtime's loader builds for that path.
    static Ptr getModel(const std::string &path_to_config_file)
    {
        return loader() ? loader()(path_to_config_file) : Ptr();
    }
    // host-runtime hook (not plugin API): the loader behind getModel
    static void setModelLoader(Loader l) { loader() = std::move(l); }

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
    // joint position limits (QPPVMPlugin.cpp:120: the JointLimits constraint's input)
    virtual bool getJointLimits(Eigen::VectorXd &q_min, Eigen::VectorXd &q_max) const
    {
        q_min.setConstant(getJointNum(), -3.14159265358979);
        q_max.setConstant(getJointNum(), 3.14159265358979);
        return true;
    }
    // XBotInterface computeJdotQdot(link, point, jdotqdot) / getPointPosition(link, point, p): the
    // bias acceleration and the position of a point given in the link frame (ForceAcc.cpp:164)
    virtual bool computeJdotQdot(const std::string &link, const Eigen::Vector3d &point, Eigen::Vector6d &jdqd) const
    {
        (void)link;
        (void)point;
        jdqd.setZero();
        return true;
    }
    bool getPointPosition(const std::string &link, const Eigen::Vector3d &point, Eigen::Vector3d &p) const
    {
        Eigen::Affine3d T;
        if (!getPose(link, T)) return false;
        p = T * point;
        return true;
    }
    bool getPose(const std::string &link, KDL::Frame &T) const
    {
        Eigen::Affine3d A;
        if (!getPose(link, A)) return false;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) T.M(r, c) = A.linear()(r, c);
            T.p(r) = A.translation()(r);
        }
        return true;
    }
    bool setJointPosition(const JointIdMap &q) { return from_map(q, &ModelInterface::getJointPosition, &ModelInterface::setJointPosition); }
    bool setJointVelocity(const JointIdMap &qd) { return from_map(qd, &ModelInterface::getJointVelocity, &ModelInterface::setJointVelocity); }
    // joint state from the robot (XBotInterface syncFrom: position and velocity)
    bool syncFrom(const RobotInterface &robot)
    {
        return robot.getMotorPosition(map_buf_) && setJointPosition(map_buf_) && robot.getMotorVelocity(map_buf_) &&
               setJointVelocity(map_buf_);
    }
    // the model's own log (XBotInterface initLog / log: joint state, one column per call)
    inline void initLog(std::shared_ptr<MatLogger> logger, int buffer_size);
    inline void log(std::shared_ptr<MatLogger> logger, double time);

private:
    Eigen::VectorXd log_buf_; // log()'s staging (sized by initLog: no allocation per call)
    static Loader &loader()
    {
        static Loader l;
        return l;
    }
    bool from_map(const JointIdMap &m, bool (ModelInterface::*get)(Eigen::VectorXd &) const,
                  bool (ModelInterface::*set)(const Eigen::VectorXd &))
    {
        (this->*get)(map_buf_);
        for (const auto &kv : m)
            if (kv.first >= 0 && kv.first < map_buf_.size()) map_buf_[kv.first] = kv.second;
        return (this->*set)(map_buf_);
    }
    Eigen::VectorXd map_buf_; // (reused: no allocation per call once sized)
};

class Handle {
public:
    using Ptr = std::shared_ptr<Handle>;
    virtual ~Handle() = default;
    virtual RobotInterface::Ptr getRobotInterface() = 0;
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

// Factory symbols XBotCore dlopens [upstream loader contract, compat form]: the named form
// (QPPVMPlugin.cpp:29) emits create_instance_<name>, the one-argument form (ForceAcc.cpp:26) one
// fixed pair per library.
#define REGISTER_XBOT_PLUGIN(plugin_name, scoped_class)                                   \
    extern "C" XBot::XBotControlPlugin *create_instance_##plugin_name() { return new scoped_class(); } \
    extern "C" void destroy_instance_##plugin_name(XBot::XBotControlPlugin *p) { delete p; }
#define REGISTER_XBOT_PLUGIN_(scoped_class)                                                \
    extern "C" XBot::XBotControlPlugin *create_instance() { return new scoped_class(); } \
    extern "C" void destroy_instance(XBot::XBotControlPlugin *p) { delete p; }

// MatLogger and the model-log members above (ModelInterface::initLog / log)
#include <XBotInterface/Logger.hpp>
