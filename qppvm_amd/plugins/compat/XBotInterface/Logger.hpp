// Logger.hpp -- compat XBot::MatLogger (XBotInterface), the logger both reference plugins use
// (QPPVMPlugin.cpp:44,54,254,258,322,325,341; ForceAcc.cpp:34,50,200,233-236,249). Same calls:
//   XBot::MatLogger::getLogger(prefix) -> Ptr, createScalarVariable / createVectorVariable
//   (name, [size,] interleave, buffer_size), add(name, scalar | vector), flush();
//   ModelInterface::initLog(logger, buffer_size) / log(logger, time) for the model's joint state.
// Each variable is a ring of buffer_size samples allocated when the variable is created: add()
// copies one sample into it and never allocates once the variable exists (the plugins create
// theirs in init_control_plugin, outside the RT loop); a full ring overwrites its oldest sample.
// flush() writes a MATLAB level-4 .mat file "<prefix>.mat" (readable by scipy.io.loadmat / MATLAB
// / Octave) with one dim x samples fp64 matrix per variable, oldest sample first. The upstream
// logger appends a timestamp to the prefix and writes MAT level 5 through matio (absent here);
// the variable names and the dim x samples layout are what a consumer of the reference's logs
// reads.
#pragma once

#include <XCM/XBotControlPlugin.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace XBot {

class MatLogger {
public:
    using Ptr = std::shared_ptr<MatLogger>;
    static constexpr int kDefaultBuffer = 10000; // samples, for variables add() creates itself

    static Ptr getLogger(const std::string &prefix) { return Ptr(new MatLogger(prefix)); }

    bool createScalarVariable(const std::string &name, int interleave = 1, int buffer_size = -1)
    {
        return createVectorVariable(name, 1, interleave, buffer_size);
    }
    bool createVectorVariable(const std::string &name, int size, int interleave = 1, int buffer_size = -1)
    {
        (void)interleave;
        if (size <= 0 || vars_.count(name)) return false;
        Var &v = vars_[name];
        v.dim = (std::size_t)size;
        v.cap = (std::size_t)(buffer_size > 0 ? buffer_size : kDefaultBuffer);
        v.data.assign(v.dim * v.cap, 0.0);
        return true;
    }

    bool add(const std::string &name, double v) { return push(name, &v, 1); }
    bool add(const std::string &name, const Eigen::VectorXd &v) { return push(name, v.data(), (std::size_t)v.size()); }
    template <int R>
    bool add(const std::string &name, const Eigen::Matrix<R, 1> &v) { return push(name, v.data(), R); }

    const std::string &path() const { return path_; }

    bool flush()
    {
        std::FILE *f = std::fopen(path_.c_str(), "wb");
        if (!f) return false;
        bool ok = true;
        for (const auto &kv : vars_) {
            const Var &v = kv.second;
            const std::size_t cols = v.count < v.cap ? v.count : v.cap;
            // MAT level 4 header: type 0000 (little-endian IEEE, fp64, full), rows, cols,
            // imaginary flag, name length incl. NUL; then the name and column-major data
            const int32_t hdr[5] = {0, (int32_t)v.dim, (int32_t)cols, 0, (int32_t)kv.first.size() + 1};
            ok = ok && std::fwrite(hdr, sizeof(hdr), 1, f) == 1;
            ok = ok && std::fwrite(kv.first.c_str(), 1, kv.first.size() + 1, f) == kv.first.size() + 1;
            // oldest sample first: the ring's head is the next slot to write
            const std::size_t head = v.count < v.cap ? 0 : v.count % v.cap;
            for (std::size_t s = 0; s < cols; ++s) {
                const double *col = v.data.data() + ((head + s) % v.cap) * v.dim;
                ok = ok && std::fwrite(col, 8, v.dim, f) == v.dim;
            }
        }
        return std::fclose(f) == 0 && ok;
    }

private:
    struct Var {
        std::size_t dim = 0, cap = 0, count = 0;
        std::vector<double> data;
    };
    explicit MatLogger(const std::string &prefix) : path_(prefix + ".mat") {}

    bool push(const std::string &name, const double *v, std::size_t dim)
    {
        auto it = vars_.find(name);
        if (it == vars_.end()) { // created on first use, as upstream (allocates: create it in init)
            createVectorVariable(name, (int)dim);
            it = vars_.find(name);
        }
        Var &var = it->second;
        if (dim != var.dim) return false; // a variable keeps its dimension
        double *dst = var.data.data() + (var.count % var.cap) * dim;
        for (std::size_t k = 0; k < dim; ++k) dst[k] = v[k];
        ++var.count;
        return true;
    }

    std::string path_;
    std::map<std::string, Var> vars_;
};

// the model's own log: joint position, velocity and effort per call, plus the time
inline void ModelInterface::initLog(MatLogger::Ptr logger, int buffer_size)
{
    const int n = getJointNum();
    for (const char *name : {"model_q", "model_qdot", "model_tau"}) logger->createVectorVariable(name, n, 1, buffer_size);
    logger->createScalarVariable("model_time", 1, buffer_size);
    log_buf_.resize(n);
}

inline void ModelInterface::log(MatLogger::Ptr logger, double time)
{
    getJointPosition(log_buf_);
    logger->add("model_q", log_buf_);
    getJointVelocity(log_buf_);
    logger->add("model_qdot", log_buf_);
    getJointEffort(log_buf_);
    logger->add("model_tau", log_buf_);
    logger->add("model_time", time);
}

}  // namespace XBot
