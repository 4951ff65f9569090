// QPPVMPlugin.h -- drop-in demo::QPPVMPlugin on the MI355X batched WBC-QP engine.
//
// Same class, namespace and XBot surface as the reference
// (include/QPPVM_RT_plugin/QPPVMPlugin.h:35-46): init_control_plugin, on_start,
// control_loop, close. What the reference delegates to OpenSoT (CartesianImpedanceCtrl x2,
// JointImpedanceCtrl, TorqueLimits, AutoStack, QPOases_sot) goes through the wbq C ABI
// (include/wbq.h); one wbq context per plugin, allocated in init_control_plugin.
#pragma once

#include <XBotInterface/Logger.hpp>
#include <XCM/XBotControlPlugin.h>

#include <cstdint>
#include <string>
#include <vector>

#include "wbq.h"

namespace demo {

class QPPVMPlugin : public XBot::XBotControlPlugin {
public:
    QPPVMPlugin();
    ~QPPVMPlugin() override;

    bool init_control_plugin(XBot::Handle::Ptr handle) override;
    void on_start(double time) override;
    void control_loop(double time, double period) override;
    bool close() override;

    // observability (the reference logs these to MatLogger: tau_qp, tau_desired)
    const Eigen::VectorXd &tau_desired() const { return _tau_d; }
    int last_status() const { return _status; }
    int last_iters() const { return _iters; } // active-set + repair steps of the last solve
    int solver_errors() const { return _solver_errors; }
    // the reference hard-codes both (QPPVMPlugin.cpp:44 "/tmp/qppvm_log", :46 _set_ref = false);
    // the dummy driver sets them before init_control_plugin / on_start
    void set_log_prefix(const std::string &prefix) { _log_prefix = prefix; }
    void set_reference_trajectory(bool on) { _set_ref = on; }
    // the JointLimits constraint the reference builds and comments out of its stack (:169-173):
    // set before init_control_plugin
    void set_joint_limits(bool on) { _use_joint_limits = on; }
    // the elbow tasks the reference builds (:154-166, on arm1_4 / arm2_4) and the stack its commented
    // line :178 closes in place of :179: ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits, no joint task
    // (include/wbq.h no_joint_task). with_joint_task = true keeps the joint task as a third level,
    // ((ee_r + ee_l) / (elbow_l + elbow_r)) / joint << limits: an extension the reference never spells.
    // Set before init_control_plugin
    void set_elbow_level(bool on, bool with_joint_task = false)
    {
        _use_elbow = on;
        _elbow_joint = with_joint_task;
    }
    int ntasks() const { return (int)_ee_links.size(); }
    const Eigen::VectorXd &joint_limit(int which) const { return which ? _q_max : _q_min; }
    const Eigen::VectorXd &joint_limit_gain(int which) const { return which ? _d_jl : _k_jl; }
    // the Cartesian references the tasks track (t = 0 right, 1 left): the on_start poses, the
    // left one replaced by the _set_ref sinusoid
    const Eigen::Affine3d &ee_reference(int t) const { return _ee_ref[t]; }

private:
    void sense();
    void syncFromMotorSide(XBot::RobotInterface::Ptr robot, XBot::ModelInterface::Ptr model);
    void QPPVMControl(const double time);

    XBot::JointIdMap _jidmap;
    XBot::RobotInterface::Ptr _robot;
    XBot::ModelInterface::Ptr _model;
    wbq_ctx *_ctx = nullptr;

    // task wiring (QPPVMPlugin.cpp:129-152): right arm then left arm, as in the stack sum; with the
    // elbow level the elbow tasks follow (:154-166: left, then right, as in :178's sum)
    std::vector<std::string> _ee_links{"arm2_7", "arm1_7"};
    bool _use_elbow = false;
    bool _elbow_joint = false;
    double _start_time = 0.0;
    int _status = 0;
    int _iters = 0;
    int _solver_errors = 0;

    Eigen::VectorXd _q, _dq, _q_ref, _q_home, _k, _d, _tau_d, _h, _tau_qp;
    Eigen::VectorXd _tau_max_const, _tau_min_const;
    std::vector<Eigen::Affine3d> _ee_ref = std::vector<Eigen::Affine3d>(2);
    // _set_ref: left end-effector reference on a circle in the y-z plane (:217-223), on the
    // reference's KDL frames (QPPVMPlugin.h:98-99)
    bool _set_ref = false;
    bool _use_joint_limits = false;
    Eigen::VectorXd _q_min, _q_max, _k_jl, _d_jl;
    KDL::Frame _start_pose;
    KDL::Frame _ref;
    std::string _log_prefix = "/tmp/qppvm_log";
    XBot::MatLogger::Ptr _matlogger;
    // per-tick input staging (instance-major, row-major: the wbq layout)
    std::vector<double> _M, _J, _pose, _pose_ref;
    Eigen::MatrixXd _Mtmp, _Jtmp;
};

}  // namespace demo
