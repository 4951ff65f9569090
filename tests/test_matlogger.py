"""The compat XBot::MatLogger (qppvm_amd/plugins/compat/XBotInterface/Logger.hpp) writes MAT
level-4 files that scipy reads back: names, dim x samples layout, values; a variable is a ring
of buffer_size samples allocated when it is created (never in add()), whose oldest samples a full
ring overwrites (CPU; g++ only)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include <XBotInterface/Logger.hpp>
int main(int argc, char **argv)
{
    auto log = XBot::MatLogger::getLogger(argv[1]);
    log->createVectorVariable("ring", 2, 1, 4); // 4 samples, then the oldest are overwritten
    Eigen::VectorXd v = Eigen::VectorXd::Zero(3);
    for (int k = 0; k < 5; ++k) {
        for (int j = 0; j < 3; ++j) v[j] = 10.0 * k + j;
        log->add("tau_qp", v);
        log->add("time_matlogger", 1e-3 * (k + 1));
    }
    Eigen::Vector3d p = Eigen::Vector3d::UnitZ();
    log->add("p", p);
    for (int k = 0; k < 7; ++k) log->add("ring", Eigen::VectorXd::Constant(2, (double)k));
    if (log->add("tau_qp", Eigen::VectorXd::Zero(2))) return 3; // a variable keeps its dimension
    return log->flush() ? 0 : 2;
}
'''


def test_matlogger_roundtrip(tmp_path):
    scipy_io = pytest.importorskip("scipy.io")
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = str(tmp_path / "t")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "qppvm_amd", "plugins", "compat"),
                           str(src), "-o", exe])
    prefix = str(tmp_path / "log")
    subprocess.check_call([exe, prefix])
    m = scipy_io.loadmat(prefix + ".mat")
    assert m["tau_qp"].shape == (3, 5)
    np.testing.assert_array_equal(m["tau_qp"], np.array([[10.0 * k + j for k in range(5)] for j in range(3)]))
    np.testing.assert_array_equal(m["time_matlogger"], 1e-3 * np.arange(1, 6)[None, :])
    np.testing.assert_array_equal(m["p"], [[0.0], [0.0], [1.0]])
    np.testing.assert_array_equal(m["ring"], np.array([[3.0, 4.0, 5.0, 6.0]] * 2))  # the last 4, oldest first
