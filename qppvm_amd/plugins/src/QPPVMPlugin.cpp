// QPPVMPlugin.cpp -- demo::QPPVMPlugin over libwbq. Mirrors the reference's control flow
// (src/QPPVMPlugin.cpp) with its own XBotInterface / Eigen / KDL spellings; the OpenSoT task
// wiring and the qpOASES solve are replaced by one wbq context and one wbq_solve per tick.
#include <QPPVM_RT_plugin/QPPVMPlugin.h>

#include <cmath>
#include <cstdio>

#include "abi_copy.h"

REGISTER_XBOT_PLUGIN(QPPVMPlugin, demo::QPPVMPlugin)

using namespace demo;

QPPVMPlugin::QPPVMPlugin() = default;

QPPVMPlugin::~QPPVMPlugin()
{
    if (_ctx) wbq_destroy(_ctx);
}

bool QPPVMPlugin::init_control_plugin(XBot::Handle::Ptr handle) // :42-199
{
    _matlogger = XBot::MatLogger::getLogger(_log_prefix); // :44
    _robot = handle->getRobotInterface();                  // :48
    // the reference hard-codes a CENTAURO yaml here (:50-51); its commented line :49 takes the
    // config the handle names, which is what a dummy-mode / test runtime can provide
    _model = XBot::ModelInterface::getModel(handle->getPathToConfigFile());
    if (!_model) return false;
    _model->initLog(_matlogger, 30000); // :54

    _model->getEffortLimits(_tau_max_const); // :56-58
    _tau_min_const = -_tau_max_const;

    _tau_d.resize(_model->getJointNum()); // :61-62
    _tau_d.setZero(_tau_d.size());
    _tau_qp.setZero(_tau_d.size());

    _model->computeNonlinearTerm(_h); // :65 (before any sync, as in the reference)

    _model->getRobotState("home", _q_home); // :69-72
    _model->setJointPosition(_q_home);
    _model->setJointVelocity(Eigen::VectorXd(_q_home.size()).setConstant(0.0));
    _model->update();

    _q = _q_home; // :74-75
    _q_ref = _q;

    // robot-side impedance: zero except the wrist joints 5-7 of both arms (:77-96)
    _k.setZero(_robot->getJointNum());
    _d.setZero(_robot->getJointNum());
    Eigen::VectorXd k0, d0;
    _robot->getStiffness(k0);
    _robot->getDamping(d0);
    for (const char *jn : {"j_arm1_5", "j_arm1_6", "j_arm1_7", "j_arm2_5", "j_arm2_6", "j_arm2_7"}) {
        const int id = _robot->getDofIndex(jn);
        if (id >= 0) {
            _k[id] = k0[id];
            _d[id] = d0[id];
        }
    }

    // task / stack / solver wiring: K = 5, D = 2 (:105-106); Kc = 700, Dc = 70 (:136-137,
    // :148-149); rows {0,1,2} (:134, :147); ((ee_right + ee_left) / joint) << limits (:177-179);
    // QPOases_sot(.., 1.0) (:188)
    const int n = _model->getJointNum();
    if (_use_elbow) _ee_links = {"arm2_7", "arm1_7", "arm1_4", "arm2_4"}; // :129-166
    const int T = (int)_ee_links.size();
    _ee_ref.resize((size_t)T);
    // the elbow tasks' gains are OpenSoT's defaults in the reference (never set, :154-166;
    // [upstream], not pinnable offline): the hands' 700 / 70 here
    const Eigen::VectorXd Kc = Eigen::VectorXd::Constant(6 * T, 700.0), Dc = Eigen::VectorXd::Constant(6 * T, 70.0);
    const Eigen::VectorXd Kq = Eigen::VectorXd::Constant(n, 5.0), Dq = Eigen::VectorXd::Constant(n, 2.0);
    wbq_desc d{};
    d.form = WBQ_FORM_QPPVM;
    d.n = n;
    d.ntasks = T;
    for (int t = 0; t < T; ++t) {
        d.row_mask[t] = 0x7;                  // OpenSoT::Indices::range(0,2) (:134, :147, :158, :165)
        d.task_level[t] = t < 2 ? 0 : 1;      // the elbows below the hands (:177-178)
    }
    // the elbow stack as the reference's commented line closes it (:177-178 in place of :179): no
    // joint task, unless the three-level extension was asked for
    d.no_joint_task = (_use_elbow && !_elbow_joint) ? 1 : 0;
    d.select_mode = WBQ_SELECT_SUBTASK;
    d.joint_weight = WBQ_WEIGHT_IDENTITY;
    d.max_batch = 1;
    d.Kc = Kc.data();
    d.Dc = Dc.data();
    d.Kq = Kq.data();
    d.Dq = Dq.data();
    d.tau_max = _tau_max_const.data();
    d.tau_min = _tau_min_const.data();
    if (_use_joint_limits) { // :120-126 and :169-171 (commented out in the reference)
        _model->getJointLimits(_q_min, _q_max);
        Eigen::VectorXd q_range = _q_max - _q_min;
        _q_max -= q_range * 0.1;
        _q_min += q_range * 0.1;
        _k_jl = k0 * 10; // _joint_limits->setGains(k0*10, d0*20)
        _d_jl = d0 * 20;
        d.joint_limits = 1;
        d.q_min = _q_min.data();
        d.q_max = _q_max.data();
        d.Kjl = _k_jl.data();
        d.Djl = _d_jl.data();
    }
    const int rc = wbq_create(&d, 0, &_ctx);
    if (rc != WBQ_SUCCESS) {
        std::fprintf(stderr, "QPPVMPlugin: wbq_create failed (%d)\n", rc);
        return false;
    }
    // the solver's log (:189, :254, :258): variables created here, outside the RT loop
    _matlogger->createVectorVariable("tau_qp", n, 1, 30000);
    _matlogger->createVectorVariable("tau_desired", n, 1, 30000);
    _matlogger->createScalarVariable("time_matlogger", 1, 30000);
    _M.resize((size_t)n * n);
    _J.resize((size_t)T * 6 * n);
    _pose.resize((size_t)12 * T);
    _pose_ref.resize((size_t)12 * T);
    return true;
}

void QPPVMPlugin::on_start(double time) // :261-305
{
    sense();
    _model->computeNonlinearTerm(_h);

    _start_time = time;
    _robot->setStiffness(_k);
    _robot->setDamping(_d);
    _robot->move();

    // references = the current poses and the current q (:271-279)
    Eigen::Affine3d left_ee_pose;
    _model->getPose(_ee_links[1], left_ee_pose);
    Eigen::Affine3d right_ee_pose;
    _model->getPose(_ee_links[0], right_ee_pose);
    _ee_ref[1] = left_ee_pose;
    _ee_ref[0] = right_ee_pose;
    for (size_t t = 2; t < _ee_links.size(); ++t) _model->getPose(_ee_links[t], _ee_ref[t]); // the elbows
    _q_ref = _q;

    _model->getPose(_ee_links[1], _start_pose); // :287
}

void QPPVMPlugin::QPPVMControl(const double time) // :201-259
{
    const int n = _model->getJointNum();
    if (_set_ref) { // :217-223 -- y += 0.15 sin(t - t0), z += 0.15 (1 - cos(t - t0)) on the left task
        _ref = _start_pose;
        _ref.p.y(_start_pose.p.y() + 0.15 * std::sin(time - _start_time));
        _ref.p.z(_start_pose.p.z() + 0.15 * (1.0 - std::cos(time - _start_time)));
        for (int r = 0; r < 3; ++r) { // _ee_task_left->setReference(_ref)
            for (int c = 0; c < 3; ++c) _ee_ref[1].linear()(r, c) = _ref.M(r, c);
            _ee_ref[1].translation()(r) = _ref.p(r);
        }
    }
    // _autostack->update(_q) (:226): the model quantities the tasks pull, copied element-wise into
    // the ABI's row-major layout (include/wbq.h; Eigen's MatrixXd is column-major)
    _model->getInertiaMatrix(_Mtmp);
    copy_row_major(_Mtmp, n, n, _M.data());
    for (int t = 0; t < (int)_ee_links.size(); ++t) {
        _model->getJacobian(_ee_links[t], _Jtmp);
        copy_row_major(_Jtmp, 6, n, _J.data() + (size_t)t * 6 * n);
        Eigen::Affine3d P;
        _model->getPose(_ee_links[t], P);
        copy_pose(P, _pose.data() + 12 * t);
        copy_pose(_ee_ref[t], _pose_ref.data() + 12 * t);
    }
    wbq_inputs in{};
    in.batch = 1;
    in.memory = WBQ_MEM_HOST;
    in.M = _M.data();
    in.J = _J.data();
    in.pose = _pose.data();
    in.pose_ref = _pose_ref.data();
    in.q = _q.data();
    in.qd = _dq.data();
    in.qref = _q_ref.data();
    in.h = _h.data();
    int32_t status = WBQ_STATUS_NUMERICAL, iters = 0;
    // solver->solve(_tau_d) (:246) and _tau_d + _h (:256) in one call: wbq returns tau = tau_qp + h
    if (wbq_set_inputs(_ctx, &in) != WBQ_SUCCESS || wbq_solve(_ctx) != WBQ_SUCCESS ||
        wbq_get_outputs(_ctx, _tau_d.data(), &status, &iters) != WBQ_SUCCESS) {
        status = WBQ_STATUS_NUMERICAL;
        _tau_d = _h;
    }
    _status = status;
    _iters = iters;
    if (status != WBQ_STATUS_OK) { // :246-249 -- tau_qp = 0, i.e. tau = h (what wbq returned)
        ++_solver_errors;
        std::fprintf(stderr, "SOLVER ERROR!\n");
    }
    _tau_qp = _tau_d;
    _tau_qp -= _h;
    _matlogger->add("tau_qp", _tau_qp);       // :254
    _matlogger->add("tau_desired", _tau_d); // :258
}

void QPPVMPlugin::control_loop(double time, double period) // :308-329
{
    (void)period;
    sense();
    _model->computeNonlinearTerm(_h);

    QPPVMControl(time);

    // set the joint effort on the model and then synchronize the effort on the robot
    _model->setJointEffort(_tau_d);
    _robot->setReferenceFrom(*_model, XBot::Sync::Effort);
    _matlogger->add("time_matlogger", time); // :322
    _model->log(_matlogger, time);           // :325
    _robot->move();
}

void QPPVMPlugin::sense() // :331-336
{
    syncFromMotorSide(_robot, _model);
    _model->getJointPosition(_q);
    _model->getJointVelocity(_dq);
}

bool QPPVMPlugin::close() // :339-342 (the reference is missing its return)
{
    if (_matlogger) _matlogger->flush();
    if (_ctx) {
        wbq_destroy(_ctx);
        _ctx = nullptr;
    }
    return true;
}

void QPPVMPlugin::syncFromMotorSide(XBot::RobotInterface::Ptr robot, XBot::ModelInterface::Ptr model) // :344-353
{
    robot->getMotorPosition(_jidmap);
    model->setJointPosition(_jidmap);

    robot->getMotorVelocity(_jidmap);
    model->setJointVelocity(_jidmap);

    model->update();
}
