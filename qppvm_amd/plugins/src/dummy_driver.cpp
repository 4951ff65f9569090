// dummy_driver.cpp -- BASELINE config 0: a plugin in an XBotCore-like dummy loop.
// init_control_plugin -> on_start -> N x control_loop (period 1 ms) -> close, on the
// synthetic robots of dummy_robot.h: the QPPVM plugin (default, n = 39 arms robot) or, with
// --plugin forceacc, the ForceAcc plugin on a floating-base quadruped (n = 30, 4 feet).
// Reports us/tick; optionally dumps the first ticks' solver inputs and outputs (binary, for
// the oracle parity tests).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <ForceAccPlugin/ForceAcc.h>
#include <QPPVM_RT_plugin/QPPVMPlugin.h>

#include "abi_copy.h"
#include "dummy_robot.h"

#include <algorithm>

// {"p50_us": .., "p99_us": ..} of the per-tick plugin times
static std::string tick_percentiles(std::vector<double> us)
{
    if (us.empty()) return "\"p50_us\": 0, \"p99_us\": 0";
    std::sort(us.begin(), us.end());
    const double p50 = us[us.size() / 2], p99 = us[std::min(us.size() - 1, (size_t)(0.99 * us.size()))];
    char buf[96];
    std::snprintf(buf, sizeof(buf), "\"p50_us\": %.3f, \"p99_us\": %.3f", p50, p99);
    return buf;
}

// ForceAcc in dummy mode: dump = header (n, nc, ticks, wrench_dim; mu as a double), then per tick
// the 13 staged solver input fields, the contact mask, tau, x and the status
static int run_forceacc(int ticks, int n, const char *dump, int dump_ticks, const char *log_prefix, int wd, double mu)
{
    auto handle = std::make_shared<dummy::Handle>(dummy::quadruped(n));
    handle->register_model();
    XBotPlugin::ForceAccExample plugin;
    if (log_prefix) plugin.set_log_prefix(log_prefix);
    plugin.set_wrench_dim(wd); // SURVEY 8f-2 (--wrench6, --mu)
    plugin.set_friction(mu);
    if (!plugin.init_control_plugin(handle)) {
        std::fprintf(stderr, "init_control_plugin failed\n");
        return 2;
    }
    FILE *f = dump ? std::fopen(dump, "wb") : nullptr;
    const double dt = 1e-3;
    {
        Eigen::VectorXd q = Eigen::VectorXd::Zero(n), qd = Eigen::VectorXd::Zero(n);
        for (int j = 0; j < n; ++j) qd[j] = 0.1 * ((j % 5) - 2);
        handle->robot().set_state(q, qd);
    }
    plugin.on_start(0.0);
    const int nc = 4;
    if (f) {
        const int hdr[4] = {n, nc, dump_ticks, plugin.wrench_dim()};
        std::fwrite(hdr, sizeof(int), 4, f);
        std::fwrite(&mu, sizeof(double), 1, f);
    }
    double worst = 0.0, run_total = 0.0;
    std::vector<double> tick_us;
    tick_us.reserve((size_t)ticks);
    int busy_ticks = 0; // ticks whose solve needed the active set or the level-0 repair
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < ticks; ++k) {
        const auto a = std::chrono::steady_clock::now();
        plugin.run((k + 1) * dt, dt);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        worst = us > worst ? us : worst;
        run_total += us;
        tick_us.push_back(us);
        busy_ticks += plugin.last_iters() > 0 ? 1 : 0;
        if (f && k < dump_ticks) {
            for (int fld = 0; fld < 13; ++fld)
                std::fwrite(plugin.staged(fld).data(), sizeof(double), plugin.staged(fld).size(), f);
            const int cm = plugin.contact_mask(), st = plugin.last_status();
            std::fwrite(&cm, sizeof(int), 1, f);
            std::fwrite(plugin.tau().data(), sizeof(double), n, f);
            std::fwrite(plugin.x().data(), sizeof(double), (size_t)plugin.x().size(), f);
            std::fwrite(&st, sizeof(int), 1, f);
        }
        // dummy-mode kinematics with the QP's acceleration (ForceAcc.cpp:225-226)
        handle->robot().step_qdd(plugin.qddot_value(), dt);
    }
    const double total = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (f) std::fclose(f);
    plugin.close();
    std::printf("{\"config\": 0, \"plugin\": \"ForceAccExample\", \"wrench_dim\": %d, \"mu\": %g, \"n\": %d, \"ticks\": %d, \"us_per_tick\": %.3f, "
                "\"run_us\": %.3f, %s, \"worst_us\": %.3f, \"busy_ticks\": %d, \"solver_errors\": %d, \"sync_flags\": %d}\n",
                plugin.wrench_dim(), mu, n, ticks, total / ticks, run_total / ticks, tick_percentiles(tick_us).c_str(), worst,
                busy_ticks, plugin.solver_errors(), handle->robot().last_sync());
    return 0;
}

int main(int argc, char **argv)
{
    int ticks = 10000, dump_ticks = 0, n = -1;
    const char *dump = nullptr;
    bool forceacc = false, stress = false, set_ref = false, joint_limits = false, elbow = false, elbow_joint = false;
    int wd = 3;
    double mu = 0.0;
    const char *log_prefix = nullptr;
    for (int k = 1; k < argc; ++k) {
        if (!std::strcmp(argv[k], "--ticks") && k + 1 < argc) ticks = std::atoi(argv[++k]);
        else if (!std::strcmp(argv[k], "--n") && k + 1 < argc) n = std::atoi(argv[++k]);
        else if (!std::strcmp(argv[k], "--plugin") && k + 1 < argc) forceacc = !std::strcmp(argv[++k], "forceacc");
        else if (!std::strcmp(argv[k], "--stress")) stress = true;
        else if (!std::strcmp(argv[k], "--set-ref")) set_ref = true; // QPPVMPlugin.cpp:217-223
        else if (!std::strcmp(argv[k], "--joint-limits")) joint_limits = true; // :169-171
        else if (!std::strcmp(argv[k], "--elbow")) elbow = true;               // :154-166, :177-178 (no joint task)
        else if (!std::strcmp(argv[k], "--elbow-joint")) elbow = elbow_joint = true; // the 3-level extension
        else if (!std::strcmp(argv[k], "--wrench6")) wd = 6;                   // ForceAcc.cpp:67
        else if (!std::strcmp(argv[k], "--mu") && k + 1 < argc) mu = std::atof(argv[++k]);
        else if (!std::strcmp(argv[k], "--log") && k + 1 < argc) log_prefix = argv[++k];
        else if (!std::strcmp(argv[k], "--dump") && k + 2 < argc) {
            dump = argv[++k];
            dump_ticks = std::atoi(argv[++k]);
        }
    }
    if (forceacc) return run_forceacc(ticks, n > 0 ? n : 30, dump, dump_ticks, log_prefix, wd, mu);
    if (n <= 0) n = 39;
    dummy::Params prm;
    prm.n = n;
    if (stress) prm.jscale = 0.5;
    const std::vector<std::string> links = elbow ? std::vector<std::string>{"arm2_7", "arm1_7", "arm1_4", "arm2_4"}
                                                 : std::vector<std::string>{"arm2_7", "arm1_7"};
    prm.links = links;
    auto handle = std::make_shared<dummy::Handle>(prm);
    handle->register_model();
    demo::QPPVMPlugin plugin;
    if (log_prefix) plugin.set_log_prefix(log_prefix);
    plugin.set_reference_trajectory(set_ref);
    plugin.set_joint_limits(joint_limits);
    plugin.set_elbow_level(elbow, elbow_joint);
    if (!plugin.init_control_plugin(handle)) {
        std::fprintf(stderr, "init_control_plugin failed\n");
        return 2;
    }
    FILE *f = dump ? std::fopen(dump, "wb") : nullptr;
    const double dt = 1e-3;
    plugin.on_start(0.0);
    if (f) {
        // header: n, ticks, tasks, then the references fixed at on_start (q_ref, pose_ref per task)
        const int hdr[3] = {n, dump_ticks, (int)links.size()};
        std::fwrite(hdr, sizeof(int), 3, f);
        Eigen::VectorXd q;
        handle->model().getJointPosition(q);
        std::fwrite(q.data(), sizeof(double), n, f);
        for (const std::string &link : links) {
            Eigen::Affine3d P;
            double pm[12];
            handle->model().getPose(link, P);
            copy_pose(P, pm);
            std::fwrite(pm, sizeof(double), 12, f);
        }
    }
    // the references are the start posture; kick the robot so the tasks have work to do
    {
        Eigen::VectorXd q = Eigen::VectorXd::Zero(n), qd = Eigen::VectorXd::Zero(n);
        for (int j = 0; j < n; ++j) qd[j] = 0.2 * ((j % 7) - 3);
        handle->robot().set_state(q, qd);
    }
    double worst = 0.0, run_total = 0.0;
    std::vector<double> tick_us;
    tick_us.reserve((size_t)ticks);
    int busy_ticks = 0; // ticks whose solve needed the active set or the level-0 repair
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < ticks; ++k) {
        const double time = (k + 1) * dt;
        const auto a = std::chrono::steady_clock::now();
        plugin.run(time, dt);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        worst = us > worst ? us : worst;
        run_total += us;
        tick_us.push_back(us);
        busy_ticks += plugin.last_iters() > 0 ? 1 : 0;
        if (f && k < dump_ticks) {
            // the solver inputs of this tick, recomputed from the (unchanged) model state
            auto &m = handle->model();
            Eigen::MatrixXd M, J;
            Eigen::VectorXd q, qd, h, tau = plugin.tau_desired();
            m.getInertiaMatrix(M);
            m.getJointPosition(q);
            m.getJointVelocity(qd);
            m.computeNonlinearTerm(h);
            std::vector<double> rm((size_t)6 * n > (size_t)n * n ? (size_t)6 * n : (size_t)n * n);
            copy_row_major(M, n, n, rm.data());
            std::fwrite(rm.data(), sizeof(double), (size_t)n * n, f);
            for (const std::string &link : links) {
                m.getJacobian(link, J);
                copy_row_major(J, 6, n, rm.data());
                std::fwrite(rm.data(), sizeof(double), (size_t)6 * n, f);
            }
            for (const std::string &link : links) {
                Eigen::Affine3d P;
                double pm[12];
                m.getPose(link, P);
                copy_pose(P, pm);
                std::fwrite(pm, sizeof(double), 12, f);
            }
            std::fwrite(q.data(), sizeof(double), n, f);
            std::fwrite(qd.data(), sizeof(double), n, f);
            std::fwrite(h.data(), sizeof(double), n, f);
            std::fwrite(tau.data(), sizeof(double), n, f);
            const int st = plugin.last_status();
            std::fwrite(&st, sizeof(int), 1, f);
        }
        handle->robot().step(handle->model(), dt); // dummy-mode physics
    }
    const double total = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (f) std::fclose(f);
    plugin.close();
    // us_per_tick: the whole loop (plugin tick + dummy model + physics); run_us: the plugin
    // tick alone (model queries, one wbq solve, torque write-back)
    std::printf("{\"config\": 0, \"plugin\": \"QPPVMPlugin\", \"plant\": \"%s\", \"n\": %d, \"ticks\": %d, \"us_per_tick\": %.3f, "
                "\"run_us\": %.3f, %s, \"worst_us\": %.3f, \"busy_ticks\": %d, \"solver_errors\": %d}\n",
                stress ? "stress (jscale 0.5, saturating)" : "nominal (jscale 0.2)", n, ticks, total / ticks,
                run_total / ticks, tick_percentiles(tick_us).c_str(), worst, busy_ticks,
                plugin.solver_errors());
    return 0;
}
