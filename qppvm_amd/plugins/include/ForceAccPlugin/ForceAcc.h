// ForceAcc.h -- drop-in XBotPlugin::ForceAccExample on the MI355X batched WBC-QP engine.
//
// Same class, namespace and XBot surface as the reference
// (include/ForceAccPlugin/ForceAcc.h:30-53): init_control_plugin, close, on_start, on_stop,
// protected control_loop. What the reference builds from OpenSoT (OptvarHelper variables
// qddot + 3 force components per foot, acceleration::Cartesian feet/waist tasks, Postural,
// DynamicFeasibility, wrench bounds, AutoStack, QPOases_sot) and the inverse-dynamics post-step
// go through the wbq contact-form C ABI (include/wbq.h, wbq_create_contact); one context per
// plugin, allocated in init_control_plugin.
#pragma once

#include <XBotInterface/Logger.hpp>
#include <XCM/XBotControlPlugin.h>

#include <cstdint>
#include <string>
#include <vector>

#include "wbq.h"

namespace XBotPlugin {

class ForceAccExample : public XBot::XBotControlPlugin {
public:
    bool init_control_plugin(XBot::Handle::Ptr handle) override;
    bool close() override;
    void on_start(double time) override;
    void on_stop(double time) override {}
    ~ForceAccExample() override;

    // observability (the reference logs tau, tau_c, qddot_value, x and the wrenches)
    const Eigen::VectorXd &tau() const { return _tau; }
    const Eigen::VectorXd &x() const { return _x; }
    const Eigen::VectorXd &qddot_value() const { return _qddot_value; }
    int last_status() const { return _status; }
    int last_iters() const { return _iters; } // active-set + repair steps of the last solve
    int solver_errors() const { return _solver_errors; }
    // the per-tick solver inputs of the last control_loop (dumped by the dummy driver)
    const std::vector<double> &staged(int field) const { return _in[field]; }
    int contact_mask() const { return _cmask; }
    // the reference hard-codes "/tmp/opensot_force_acc_example" (ForceAcc.cpp:34)
    void set_log_prefix(const std::string &prefix) { _log_prefix = prefix; }
    // SURVEY 8f-2 options, set before init_control_plugin: 6 = the full-wrench variables the
    // reference comments on ("put 6 for full wrench", ForceAcc.cpp:67; its 6-D box :74-76);
    // mu > 0 = the linearised friction pyramid (no cone in the reference)
    void set_wrench_dim(int wd) { _wd = wd == 6 ? 6 : 3; }
    void set_friction(double mu) { _mu = mu; }
    int wrench_dim() const { return _wd; }

protected:
    void control_loop(double time, double period) override;

private:
    void sync_model();

    XBot::RobotInterface::Ptr _robot;
    XBot::ModelInterface::Ptr _model;
    wbq_ctx *_ctx = nullptr;

    double _start_time = 0.0;
    int _status = 0;
    int _iters = 0;
    int _solver_errors = 0;
    int _cmask = 0xF;
    int _wd = 3;       // variables per contact: 3 forces (:67) or the 6-D wrench
    double _mu = 0.0;  // friction pyramid coefficient (0: none, the reference)

    Eigen::VectorXd _k, _d, _q, _qdot, _q_ref, _tau, _tau_c, _x, _qddot_value, _h;
    Eigen::Vector3d _initial_com; // ForceAcc.h:69 (the pelvis origin, ForceAcc.cpp:164)
    Eigen::MatrixXd _Mtmp, _Jtmp;
    std::vector<Eigen::VectorXd> _wrench_value; // [f_c; 0] (or the 6-D wrench) per contact (ForceAcc.cpp:61,199)
    Eigen::Affine3d _waist_ref;
    std::vector<Eigen::Affine3d> _feet_ref;
    std::vector<std::string> _contact_links{"foot_fl", "foot_fr", "foot_hr", "foot_hl"}; // ForceAcc.cpp:58
    std::string _waist_link = "pelvis";                                                   // :29
    // staged wbq_contact_inputs fields (M, h, q, qd, qref, Jw, jdqd_w, pose_w, pose_w_ref,
    // Jc, jdqd_c, pose_c, pose_c_ref), one instance
    std::vector<double> _in[13];
    std::string _log_prefix = "/tmp/opensot_force_acc_example";
    XBot::MatLogger::Ptr _logger;
};

}  // namespace XBotPlugin
