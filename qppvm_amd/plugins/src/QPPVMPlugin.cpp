// QPPVMPlugin.cpp -- demo::QPPVMPlugin over libwbq. Mirrors the reference's control flow
// (src/QPPVMPlugin.cpp), with the OpenSoT/qpOASES solve replaced by one wbq_solve.
#include <QPPVM_RT_plugin/QPPVMPlugin.h>

#include <cmath>
#include <cstdio>
#include <cstring>

#include "abi_copy.h"

REGISTER_XBOT_PLUGIN(QPPVMPlugin, demo::QPPVMPlugin)

using namespace demo;

QPPVMPlugin::QPPVMPlugin() = default;

QPPVMPlugin::~QPPVMPlugin()
{
    if (_ctx) wbq_destroy(_ctx);
}

bool QPPVMPlugin::init_control_plugin(XBot::Handle::Ptr handle)
{
    _robot = handle->getRobotInterface();
    _matlogger = XBot::MatLogger::getLogger(_log_prefix); // :44
    _model = handle->getModel(); // reference: hard-coded CENTAURO yaml (:50-51)
    const int n = _model->getJointNum();
    _matlogger->reserve(30000); // _model->initLog(_matlogger, 30000) (:54)

    _model->getEffortLimits(_tau_max_const); // :56-58
    _tau_min_const.setZero(n);
    for (int j = 0; j < n; ++j) _tau_min_const[j] = -_tau_max_const[j];
    _tau_d.setZero(n);
    _model->computeNonlinearTerm(_h); // :65 (before any sync, as in the reference)

    _model->getRobotState("home", _q_home); // :69-72
    _model->setJointPosition(_q_home);
    _model->setJointVelocity(Eigen::VectorXd(n, 0.0));
    _model->update();
    _q = _q_home;
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
    // :148-149); rows {0,1,2} (:134, :147); ((ee_right + ee_left) / joint) << limits (:177)
    std::vector<double> Kc(12, 700.0), Dc(12, 70.0), Kq(n, 5.0), Dq(n, 2.0);
    wbq_desc d{};
    d.form = WBQ_FORM_QPPVM;
    d.n = n;
    d.ntasks = 2;
    d.row_mask[0] = d.row_mask[1] = 0x7;
    d.select_mode = WBQ_SELECT_SUBTASK;
    d.joint_weight = WBQ_WEIGHT_IDENTITY;
    d.max_batch = 1;
    d.Kc = Kc.data();
    d.Dc = Dc.data();
    d.Kq = Kq.data();
    d.Dq = Dq.data();
    d.tau_max = _tau_max_const.data();
    d.tau_min = _tau_min_const.data();
    const int rc = wbq_create(&d, 0, &_ctx);
    if (rc != WBQ_SUCCESS) {
        std::fprintf(stderr, "QPPVMPlugin: wbq_create failed (%d)\n", rc);
        return false;
    }
    _M.resize((size_t)n * n);
    _J.resize((size_t)2 * 6 * n);
    _pose.resize(24);
    _pose_ref.resize(24);
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
    // references = current poses and current q (:271-279)
    for (int t = 0; t < 2; ++t) _model->getPose(_ee_links[t], _ref[t]);
    _q_ref = _q;
    _model->getPose(_ee_links[1], _start_pose); // left end effector (:284)
}

void QPPVMPlugin::QPPVMControl(double time) // :201-259
{
    const int n = _model->getJointNum();
    if (_set_ref) { // :217-223 -- y += 0.15 sin(t - t0), z += 0.15 (1 - cos(t - t0)) on the left task
        _ref[1] = _start_pose;
        _ref[1].m[7] = _start_pose.m[7] + 0.15 * std::sin(time - _start_time);
        _ref[1].m[11] = _start_pose.m[11] + 0.15 * (1.0 - std::cos(time - _start_time));
    }
    Eigen::MatrixXd M, J;
    // element-wise into the ABI's row-major layout (include/wbq.h): Eigen's MatrixXd is
    // column-major, so its data() is never copied as is
    _model->getInertiaMatrix(M);
    copy_row_major(M, n, n, _M.data());
    for (int t = 0; t < 2; ++t) {
        _model->getJacobian(_ee_links[t], J);
        copy_row_major(J, 6, n, _J.data() + (size_t)t * 6 * n);
        Eigen::Affine3d P;
        _model->getPose(_ee_links[t], P);
        std::memcpy(_pose.data() + 12 * t, P.m, sizeof(P.m));
        std::memcpy(_pose_ref.data() + 12 * t, _ref[t].m, sizeof(P.m));
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
    int32_t status = 3, iters = 0;
    _tau_d.setZero(n);
    if (wbq_set_inputs(_ctx, &in) != WBQ_SUCCESS || wbq_solve(_ctx) != WBQ_SUCCESS ||
        wbq_get_outputs(_ctx, _tau_d.data(), &status, &iters) != WBQ_SUCCESS) {
        status = WBQ_STATUS_NUMERICAL;
        for (int j = 0; j < n; ++j) _tau_d[j] = _h[j];
    }
    _status = status;
    _iters = iters;
    if (status != WBQ_STATUS_OK) { // :246-249 -- tau_qp = 0, i.e. tau = h (already in tau)
        ++_solver_errors;
        std::fprintf(stderr, "SOLVER ERROR!\n");
    }
    Eigen::VectorXd tau_qp(n, 0.0);
    for (int j = 0; j < n; ++j) tau_qp[j] = _tau_d[j] - _h[j];
    _matlogger->add("tau_qp", tau_qp);       // :254
    _matlogger->add("tau_desired", _tau_d); // :258
}

void QPPVMPlugin::control_loop(double time, double /*period*/) // :308-329
{
    sense();
    _model->computeNonlinearTerm(_h);
    QPPVMControl(time);
    _model->setJointEffort(_tau_d);
    _robot->setReferenceFrom(*_model, XBot::Sync::Effort);
    _matlogger->add("time_matlogger", time); // :322
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

void QPPVMPlugin::syncFromMotorSide(XBot::RobotInterface::Ptr robot, XBot::ModelInterface::Ptr model)
{
    Eigen::VectorXd v;
    robot->getMotorPosition(v);
    model->setJointPosition(v);
    robot->getMotorVelocity(v);
    model->setJointVelocity(v);
    model->update();
}
