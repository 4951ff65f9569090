// ForceAcc.cpp -- XBotPlugin::ForceAccExample over libwbq. Mirrors the reference's control
// flow (src/ForceAcc.cpp), with the OpenSoT/qpOASES solve and the inverse-dynamics
// post-step replaced by one wbq_solve of the contact form.
#include <ForceAccPlugin/ForceAcc.h>

#include <cstdio>
#include <cstring>

#include "abi_copy.h"

REGISTER_XBOT_PLUGIN(ForceAccExample, XBotPlugin::ForceAccExample)

using namespace XBotPlugin;

ForceAccExample::~ForceAccExample()
{
    if (_ctx) wbq_destroy(_ctx);
}

bool ForceAccExample::init_control_plugin(XBot::Handle::Ptr handle) // :31-141
{
    _robot = handle->getRobotInterface();
    _logger = XBot::MatLogger::getLogger(_log_prefix); // :34
    _logger->reserve(10000);                           // _model->initLog(_logger, 10000) (:50)
    _robot->getStiffness(_k); // :36-39: impedance / 16, damping / 4
    _robot->getDamping(_d);
    for (size_t j = 0; j < _k.size(); ++j) {
        _k[j] /= 16.0;
        _d[j] /= 4.0;
    }
    _model = handle->getModel(); // reference: getModel(handle->getPathToConfigFile()) :43
    const int n = _model->getJointNum();
    Eigen::VectorXd qhome;
    _model->getRobotState("home", qhome); // :45-48
    _model->setJointPosition(qhome);
    _model->update();

    // stack wiring (:58-137): x = [qddot; f_c x 4], wrench bounds (-1000,-1000,10)..(1000,..),
    // waist / (postural + feet) << dyn_feas << wrench bounds; the acceleration-task gains are
    // OpenSoT defaults upstream, here the build's named defaults (critically damped, Kp = 1)
    wbq_contact_desc d{};
    d.n = n;
    d.n_fb = 6;
    d.nc = (int)_contact_links.size();
    d.torque_rows = 0; // the reference stack has no torque-limit rows (:131-133)
    d.max_batch = 1;
    d.Kp_w = d.Kp_f = d.Kp_p = 1.0;
    d.Kd_w = d.Kd_f = d.Kd_p = 2.0;
    const double lb[3] = {-1000.0, -1000.0, 10.0}, ub[3] = {1000.0, 1000.0, 1000.0}; // :74-76
    for (int k = 0; k < 3; ++k) {
        d.f_lb[k] = lb[k];
        d.f_ub[k] = ub[k];
    }
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
    _x.setZero(n + 3 * nc);
    _tau.setZero(n);
    _qddot_value.setZero(n);
    return true;
}

void ForceAccExample::on_start(double time) // :150-165
{
    _start_time = time;
    sync_model();
    _model->getJointPosition(_q);
    _q_ref = _q; // postural reference: the start posture
    for (size_t c = 0; c < _contact_links.size(); ++c) _model->getPose(_contact_links[c], _feet_ref[c]); // resetReference
    _model->getPose(_waist_link, _waist_ref);
    _model->getPointPosition(_waist_link, _initial_com); // :164 ("com" is the pelvis origin)
}

void ForceAccExample::control_loop(double /*time*/, double /*period*/) // :167-253
{
    sync_model();
    const int n = _model->getJointNum();
    const size_t nc = _contact_links.size();
    // waist reference: p_init - 0.1 z, orientation as at start (:181)
    for (int k = 0; k < 3; ++k) _waist_ref.m[4 * k + 3] = _initial_com[k] - (k == 2 ? 0.1 : 0.0);

    Eigen::MatrixXd M, J;
    Eigen::VectorXd v;
    Eigen::Affine3d P;
    _model->getInertiaMatrix(M);
    copy_row_major(M, n, n, _in[0].data()); // element-wise: Eigen's MatrixXd is column-major
    _model->computeNonlinearTerm(_h);
    std::memcpy(_in[1].data(), _h.data(), sizeof(double) * n);
    _model->getJointPosition(_q);
    _model->getJointVelocity(_qdot);
    std::memcpy(_in[2].data(), _q.data(), sizeof(double) * n);
    std::memcpy(_in[3].data(), _qdot.data(), sizeof(double) * n);
    std::memcpy(_in[4].data(), _q_ref.data(), sizeof(double) * n);
    _model->getJacobian(_waist_link, J);
    copy_row_major(J, 6, n, _in[5].data());
    _model->computeJdotQdot(_waist_link, v);
    std::memcpy(_in[6].data(), v.data(), sizeof(double) * 6);
    _model->getPose(_waist_link, P);
    std::memcpy(_in[7].data(), P.m, sizeof(P.m));
    std::memcpy(_in[8].data(), _waist_ref.m, sizeof(P.m));
    for (size_t c = 0; c < nc; ++c) {
        _model->getJacobian(_contact_links[c], J);
        copy_row_major(J, 6, n, _in[9].data() + c * 6 * n);
        _model->computeJdotQdot(_contact_links[c], v);
        std::memcpy(_in[10].data() + c * 6, v.data(), sizeof(double) * 6);
        _model->getPose(_contact_links[c], P);
        std::memcpy(_in[11].data() + c * 12, P.m, sizeof(P.m));
        std::memcpy(_in[12].data() + c * 12, _feet_ref[c].m, sizeof(P.m));
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
    int32_t status = WBQ_STATUS_NUMERICAL, iters = 0;
    Eigen::VectorXd tau(n, 0.0);
    if (wbq_set_contact_inputs(_ctx, &in) != WBQ_SUCCESS || wbq_solve(_ctx) != WBQ_SUCCESS ||
        wbq_get_outputs(_ctx, tau.data(), &status, &iters) != WBQ_SUCCESS ||
        wbq_get_contact_outputs(_ctx, _x.data()) != WBQ_SUCCESS)
        status = WBQ_STATUS_NUMERICAL;
    _status = status;
    _iters = iters;
    if (status != WBQ_STATUS_OK) { // :189-193: "Unable to solve!!!", no command this tick
        ++_solver_errors;
        std::fprintf(stderr, "Unable to solve!!!\n");
        return;
    }
    for (int j = 0; j < n; ++j) _qddot_value[j] = _x[j]; // :196
    _tau = tau;                                          // ID(q, qd, qdd) - tau_c (:206-218)
    // logs (:200, :233-236): wrench w_c = [f_c; 0] per contact, tau_c = sum_c J_c^T w_c
    Eigen::VectorXd tau_c(n, 0.0), w(6, 0.0);
    for (size_t c = 0; c < nc; ++c) {
        for (int k = 0; k < 3; ++k) w[k] = _x[n + 3 * c + k];
        const double *Jc = _in[9].data() + c * 6 * n; // row-major 6 x n
        for (int k = 0; k < 3; ++k)
            for (int j = 0; j < n; ++j) tau_c[j] += Jc[k * n + j] * w[k];
        _logger->add(_contact_links[c] + "_wrench", w);
    }
    _logger->add("tau", _tau);
    _logger->add("tau_c", tau_c);
    _logger->add("qddot_value", _qddot_value);
    _logger->add("x", _x);
    _model->setJointEffort(_tau);                        // :219
    _robot->setStiffness(_k);                            // :239-241 (re-sent every tick)
    _robot->setDamping(_d);
    _robot->setReferenceFrom(*_model, XBot::Sync::Position, XBot::Sync::Effort); // :242
    _robot->move(); // :248
}

void ForceAccExample::sync_model() // :256-282; floating-base state comes with the model here
{
    Eigen::VectorXd v;
    _robot->getMotorPosition(v);
    _model->setJointPosition(v);
    _robot->getMotorVelocity(v);
    _model->setJointVelocity(v);
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
