// ForceAcc.cpp -- XBotPlugin::ForceAccExample over libwbq. Mirrors the reference's control
// flow (src/ForceAcc.cpp) with its own XBotInterface / Eigen spellings; the OpenSoT stack, the
// qpOASES solve and the inverse-dynamics post-step are replaced by one wbq_solve of the contact
// form.
#include <ForceAccPlugin/ForceAcc.h>

#include <cstdio>
#include <cstring>

#include "abi_copy.h"

/* Specify that the class XBotPlugin::ForceAccExample is a XBot RT plugin (ForceAcc.cpp:26) */
REGISTER_XBOT_PLUGIN_(XBotPlugin::ForceAccExample)

using namespace XBotPlugin;

ForceAccExample::~ForceAccExample()
{
    if (_ctx) wbq_destroy(_ctx);
}

bool ForceAccExample::init_control_plugin(XBot::Handle::Ptr handle) // :31-141
{
    _robot = handle->getRobotInterface();
    _logger = XBot::MatLogger::getLogger(_log_prefix); // :34

    _robot->getStiffness(_k); // :36-39: impedance / 16, damping / 4
    _robot->getDamping(_d);
    _k /= 16;
    _d /= 4;

    _model = XBot::ModelInterface::getModel(handle->getPathToConfigFile()); // :43
    if (!_model) return false;

    Eigen::VectorXd qhome; // :45-48
    _model->getRobotState("home", qhome);
    _model->setJointPosition(qhome);
    _model->update();

    _model->initLog(_logger, 10000); // :50

    // stack wiring (:58-137): x = [qddot; f_c x 4], wrench bounds (-1000,-1000,10)..(1000,..),
    // (with set_wrench_dim(6): x = [qddot; w_c x 4] boxed by the full 6-D bounds)
    // waist / (postural + feet) << dyn_feas << wrench bounds; the acceleration-task gains are
    // OpenSoT defaults upstream, here the build's named defaults (critically damped, Kp = 1)
    const int n = _model->getJointNum();
    _wrench_value.assign(_contact_links.size(), Eigen::VectorXd::Zero(6)); // :61
    wbq_contact_desc d{};
    d.n = n;
    d.n_fb = 6;
    d.nc = (int)_contact_links.size();
    d.torque_rows = 0; // the reference stack has no torque-limit rows (:131-133)
    d.max_batch = 1;
    d.Kp_w = d.Kp_f = d.Kp_p = 1.0;
    d.Kd_w = d.Kd_f = d.Kd_p = 2.0;
    Eigen::VectorXd wrench_ub(6), wrench_lb(6); // :74-76
    wrench_ub << 1000, 1000, 1000, 1, 1, 1;
    wrench_lb << -1000, -1000, 10, -1, -1, -1;
    for (int k = 0; k < 3; ++k) {
        d.f_lb[k] = wrench_lb[k];
        d.f_ub[k] = wrench_ub[k];
        d.m_lb[k] = wrench_lb[3 + k]; // bound only with the full wrench (wrench_dim 6)
        d.m_ub[k] = wrench_ub[3 + k];
    }
    d.wrench_dim = _wd; // :67 vars.emplace_back(cl, 3) -- "put 6 for full wrench"
    d.mu = _mu;
    d.eps_f = 1e-8; // explicit min-norm tie-break of the internal forces
    const int rc = wbq_create_contact(&d, 0, &_ctx);
    if (rc != WBQ_SUCCESS) {
        std::fprintf(stderr, "ForceAccExample: wbq_create_contact failed (%d)\n", rc);
        return false;
    }
    const size_t nc = _contact_links.size();
    const size_t sizes[13] = {(size_t)n * n, (size_t)n, (size_t)n, (size_t)n, (size_t)n, 6 * (size_t)n, 6, 12, 12,
                              nc * 6 * n, nc * 6, nc * 12, nc * 12};
    for (int f = 0; f < 13; ++f) _in[f].assign(sizes[f], 0.0);
    _feet_ref.resize(nc);
    _x.setZero(n + _wd * (int)nc);
    _tau.setZero(n);
    _tau_c.setZero(n);
    _qddot_value.setZero(n);
    // the plugin's log (:200, :233-236): variables created here, outside the RT loop
    for (const auto &cl : _contact_links) _logger->createVectorVariable(cl + "_wrench", 6, 1, 10000);
    _logger->createVectorVariable("tau", n, 1, 10000);
    _logger->createVectorVariable("tau_c", n, 1, 10000);
    _logger->createVectorVariable("qddot_value", n, 1, 10000);
    _logger->createVectorVariable("x", n + _wd * (int)nc, 1, 10000);
    return true;
}

void ForceAccExample::on_start(double time) // :143-165
{
    _start_time = time;
    sync_model();
    _model->getJointPosition(_q);
    _q_ref = _q; // postural reference: the start posture
    // resetReference of the feet and waist tasks (:157-162): the current poses
    for (size_t c = 0; c < _contact_links.size(); ++c) _model->getPose(_contact_links[c], _feet_ref[c]);
    _model->getPose(_waist_link, _waist_ref);
    _model->getPointPosition(_waist_link, Eigen::Vector3d::Zero(), _initial_com); // :164
}

void ForceAccExample::control_loop(double time, double period) // :167-253
{
    (void)period;
    sync_model(); // :172-178
    const int n = _model->getJointNum();
    const size_t nc = _contact_links.size();

    /* Set reference (:181): the pelvis 10 cm below its start position, orientation as at start */
    _waist_ref.translation() = _initial_com - 0.1 * Eigen::Vector3d::UnitZ();

    /* Update stack (:184): the model quantities the tasks and constraints pull, element-wise into
     * the ABI's row-major layout (Eigen's MatrixXd is column-major) */
    Eigen::Vector6d jdqd;
    Eigen::Affine3d P;
    _model->getInertiaMatrix(_Mtmp);
    copy_row_major(_Mtmp, n, n, _in[0].data());
    _model->computeNonlinearTerm(_h);
    std::memcpy(_in[1].data(), _h.data(), sizeof(double) * n);
    _model->getJointPosition(_q);
    _model->getJointVelocity(_qdot);
    std::memcpy(_in[2].data(), _q.data(), sizeof(double) * n);
    std::memcpy(_in[3].data(), _qdot.data(), sizeof(double) * n);
    std::memcpy(_in[4].data(), _q_ref.data(), sizeof(double) * n);
    _model->getJacobian(_waist_link, _Jtmp);
    copy_row_major(_Jtmp, 6, n, _in[5].data());
    _model->computeJdotQdot(_waist_link, Eigen::Vector3d::Zero(), jdqd);
    std::memcpy(_in[6].data(), jdqd.data(), sizeof(double) * 6);
    _model->getPose(_waist_link, P);
    copy_pose(P, _in[7].data());
    copy_pose(_waist_ref, _in[8].data());
    for (size_t c = 0; c < nc; ++c) {
        _model->getJacobian(_contact_links[c], _Jtmp);
        copy_row_major(_Jtmp, 6, n, _in[9].data() + c * 6 * n);
        _model->computeJdotQdot(_contact_links[c], Eigen::Vector3d::Zero(), jdqd);
        std::memcpy(_in[10].data() + c * 6, jdqd.data(), sizeof(double) * 6);
        _model->getPose(_contact_links[c], P);
        copy_pose(P, _in[11].data() + c * 12);
        copy_pose(_feet_ref[c], _in[12].data() + c * 12);
    }
    wbq_contact_inputs in{};
    in.batch = 1;
    in.memory = WBQ_MEM_HOST;
    in.M = _in[0].data();
    in.h = _in[1].data();
    in.q = _in[2].data();
    in.qd = _in[3].data();
    in.qref = _in[4].data();
    in.Jw = _in[5].data();
    in.jdqd_w = _in[6].data();
    in.pose_w = _in[7].data();
    in.pose_w_ref = _in[8].data();
    in.Jc = _in[9].data();
    in.jdqd_c = _in[10].data();
    in.pose_c = _in[11].data();
    in.pose_c_ref = _in[12].data();
    const int32_t cm = _cmask;
    in.cmask = &cm;

    /* Solve QP (:188-193) and the ID post-step tau = M qdd + h - sum_c J_c^T w_c (:206-218) */
    int32_t status = WBQ_STATUS_NUMERICAL, iters = 0;
    _x.setZero(_x.size());
    if (wbq_set_contact_inputs(_ctx, &in) != WBQ_SUCCESS || wbq_solve(_ctx) != WBQ_SUCCESS ||
        wbq_get_outputs(_ctx, _tau.data(), &status, &iters) != WBQ_SUCCESS ||
        wbq_get_contact_outputs(_ctx, _x.data()) != WBQ_SUCCESS)
        status = WBQ_STATUS_NUMERICAL;
    _status = status;
    _iters = iters;
    if (status != WBQ_STATUS_OK) { // :189-193: "Unable to solve!!!", no command this tick
        ++_solver_errors;
        std::fprintf(stderr, "Unable to solve!!!\n");
        return;
    }

    /* Retrieve values (:196-201) */
    for (int j = 0; j < n; ++j) _qddot_value[j] = _x[j];
    for (size_t i = 0; i < nc; i++) {
        for (int k = 0; k < _wd; ++k) _wrench_value[i][k] = _x[n + _wd * i + k];
        _logger->add(_contact_links[i] + "_wrench", _wrench_value[i]);
    }

    /* Compute torques due to contacts (:206-210), for the log: tau_c = sum_i J_i^T w_i */
    _tau_c.setZero(_model->getJointNum());
    for (size_t i = 0; i < nc; i++) {
        const double *Jc = _in[9].data() + i * 6 * n; // row-major 6 x n
        for (int k = 0; k < _wd; ++k)
            for (int j = 0; j < n; ++j) _tau_c[j] += Jc[k * n + j] * _wrench_value[i][k];
    }
    _model->setJointEffort(_tau); // :219

    _logger->add("tau", _tau); // :233-236
    _logger->add("tau_c", _tau_c);
    _logger->add("qddot_value", _qddot_value);
    _logger->add("x", _x);

    /* Send commands to robot (:239-248) */
    _robot->setStiffness(_k);
    _robot->setDamping(_d);
    _robot->setReferenceFrom(*_model, XBot::Sync::Position, XBot::Sync::Effort);
    _robot->move();
    _model->log(_logger, time); // :249
}

void ForceAccExample::sync_model() // :256-282; the floating-base state comes with the robot state here
{
    _model->syncFrom(*_robot);
    _model->update();
}

bool ForceAccExample::close() // ForceAcc.h:43
{
    if (_logger) _logger->flush();
    if (_ctx) {
        wbq_destroy(_ctx);
        _ctx = nullptr;
    }
    return true;
}
