"""The plugin boundary speaks the reference's API: the compat XCM /
XBotInterface / Eigen / KDL header (qppvm_amd/plugins/compat) accepts the reference plugins' own
call spellings and rejects the ones real Eigen / XBotInterface reject, and the plugin shells use
nothing the real libraries lack. CPU only (g++ -fsyntax-only)."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(ROOT, "qppvm_amd", "plugins", "compat")
SHELLS = [os.path.join(ROOT, "qppvm_amd", "plugins", "src", f) for f in ("QPPVMPlugin.cpp", "ForceAcc.cpp")] + [
    os.path.join(ROOT, "qppvm_amd", "plugins", "include", d, f)
    for d, f in (("QPPVM_RT_plugin", "QPPVMPlugin.h"), ("ForceAccPlugin", "ForceAcc.h"))]


def _compile(body: str) -> subprocess.CompletedProcess:
    src = "#include <XCM/XBotControlPlugin.h>\n#include <XBotInterface/Logger.hpp>\n#include <cmath>\n" + body
    with tempfile.NamedTemporaryFile("w", suffix=".cpp", delete=False) as f:
        f.write(src)
        path = f.name
    try:
        return subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", COMPAT, path], capture_output=True, text=True)
    finally:
        os.unlink(path)


# the reference's spellings: QPPVMPlugin.cpp:44-75,203-204,217-222,256,271-287,344-353;
# ForceAcc.cpp:36-50,61,74-76,164,181,188,196-210,249 (OpenSoT calls excluded: the wbq C ABI replaces them)
REFERENCE_SNIPPET = r'''
struct Snippet {
    XBot::RobotInterface::Ptr _robot;
    XBot::ModelInterface::Ptr _model;
    XBot::MatLogger::Ptr _matlogger;
    XBot::JointIdMap _jidmap;
    Eigen::VectorXd _tau_max_const, _tau_min_const, _tau_d, _h, _tau_max, _q_home, _q, _k, _d, _x;
    KDL::Frame _start_pose, _ref;
    Eigen::Vector3d _initial_com;
    std::vector<Eigen::VectorXd> _wrench_value;
    double _start_time = 0.0;
    void qppvm(XBot::Handle::Ptr handle, double time) {
        _matlogger = XBot::MatLogger::getLogger("/tmp/qppvm_log");
        _robot = handle->getRobotInterface();
        _model = XBot::ModelInterface::getModel(handle->getPathToConfigFile());
        _model->initLog(_matlogger, 30000);
        _model->getEffortLimits(_tau_max_const);
        _tau_min_const = -_tau_max_const;
        _tau_d.resize(_model->getJointNum());
        _tau_d.setZero(_tau_d.size());
        _model->computeNonlinearTerm(_h);
        _tau_max = _tau_max_const - _h;
        _model->getRobotState("home", _q_home);
        _model->setJointPosition(_q_home);
        _model->setJointVelocity(Eigen::VectorXd(_q_home.size()).setConstant(0.0));
        _model->update();
        _k.setZero(_robot->getJointNum());
        Eigen::VectorXd k0;
        _robot->getStiffness(k0);
        _k[_robot->getDofIndex("j_arm1_5")] = k0[_robot->getDofIndex("j_arm1_5")];
        Eigen::Affine3d left_ee_pose;
        _model->getPose("arm1_7", left_ee_pose);
        Eigen::Matrix4d ref = left_ee_pose.matrix();
        (void)ref;
        _model->getPose("arm1_7", _start_pose);
        _ref = _start_pose;
        _ref.p.y(_start_pose.p.y() + 0.15 * std::sin(time - _start_time));
        _ref.p.z(_start_pose.p.z() + 0.15 * (1.0 - std::cos(time - _start_time)));
        _tau_d.setZero(_tau_d.size());
        _matlogger->add("tau_qp", _tau_d);
        _tau_d = _tau_d + _h;
        _model->setJointEffort(_tau_d);
        _robot->setReferenceFrom(*_model, XBot::Sync::Effort);
        _matlogger->add("time_matlogger", time);
        _model->log(_matlogger, time);
        _robot->move();
        _robot->getMotorPosition(_jidmap);
        _model->setJointPosition(_jidmap);
        _robot->getMotorVelocity(_jidmap);
        _model->setJointVelocity(_jidmap);
        _matlogger->flush();
    }
    void forceacc(XBot::Handle::Ptr handle, double time) {
        _robot = handle->getRobotInterface();
        _robot->getStiffness(_k);
        _robot->getDamping(_d);
        _k /= 16;
        _d /= 4;
        _model = XBot::ModelInterface::getModel(handle->getPathToConfigFile());
        Eigen::VectorXd qhome;
        _model->getRobotState("home", qhome);
        _model->initLog(_matlogger, 10000);
        _wrench_value.assign(4, Eigen::VectorXd::Zero(6));
        _model->getPointPosition("pelvis", Eigen::Vector3d::Zero(), _initial_com);
        Eigen::Vector3d waist_ref = _initial_com - 0.1 * Eigen::Vector3d::UnitZ();
        (void)waist_ref;
        _x.setZero(_x.size());
        _matlogger->add("foot_fl_wrench", _wrench_value[0]);
        _model->syncFrom(*_robot);
        Eigen::Affine3d w_T_fb;
        Eigen::Matrix3d w_R_fb;
        Eigen::Vector3d fb_pos;
        Eigen::Vector6d fb_twist;
        w_T_fb.linear() = w_R_fb;
        w_T_fb.translation() = fb_pos;
        (void)fb_twist;
        _robot->setReferenceFrom(*_model, XBot::Sync::Position, XBot::Sync::Effort);
        _model->log(_matlogger, time);
        Eigen::VectorXd wrench_ub(6), wrench_lb(6);   // ForceAcc.cpp:74-76
        wrench_ub << 1000, 1000, 1000, 1, 1, 1;
        wrench_lb << -1000, -1000, 10, -1, -1, -1;
        (void)wrench_ub;
    }
};
'''


def test_reference_spellings_compile():
    r = _compile(REFERENCE_SNIPPET)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("body", [
    "void f() { Eigen::VectorXd v(6, 0.0); }",                                 # Eigen: no (size, value) ctor
    "void f() { Eigen::Affine3d T; double x = T.m[3]; (void)x; }",            # Eigen: no raw member
    "void f(XBot::Handle::Ptr h) { auto m = h->getModel(); (void)m; }",        # XCM: getModel is static
])
def test_compat_only_spellings_rejected(body):
    assert _compile(body).returncode != 0


def test_shells_use_no_compat_only_api():
    bad = [r"\.m\[", r"VectorXd\s*\w*\s*\(\s*[^()]*,\s*0\.0\s*\)", r"handle->getModel\(\)", r"->reserve\("]
    for path in SHELLS:
        text = open(path).read()
        for pat in bad:
            assert not re.search(pat, text), (path, pat)
    # both shells take their model the reference's way (QPPVMPlugin.cpp:50, ForceAcc.cpp:43)
    for path in SHELLS[:2]:
        assert "XBot::ModelInterface::getModel(handle->getPathToConfigFile())" in open(path).read(), path
