// Logger.hpp -- compat XBot::MatLogger (XBotInterface), the logger both reference plugins use
// (QPPVMPlugin.cpp:44,254,258,322,341; ForceAcc.cpp:34,200,233-236). Same calls:
//   XBot::MatLogger::getLogger(prefix) -> Ptr, add(name, scalar | vector), flush().
// Samples are kept in memory, one column per add(); flush() writes a MATLAB level-4 .mat
// file "<prefix>.mat" (readable by scipy.io.loadmat / MATLAB / Octave) with one dim x samples
// fp64 matrix per variable, named as logged. The upstream logger appends a timestamp to the
// prefix and writes MAT level 5 through matio (absent here); the variable names and the
// dim x samples layout are what a consumer of the reference's logs reads.
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

    static Ptr getLogger(const std::string &prefix) { return Ptr(new MatLogger(prefix)); }

    // capacity hint (samples per variable), as ModelInterface::initLog(logger, buffer_size)
    void reserve(std::size_t samples) { reserve_ = samples; }

    bool add(const std::string &name, double v) { return push(name, &v, 1); }
    bool add(const std::string &name, const Eigen::VectorXd &v) { return push(name, v.data(), v.size()); }

    const std::string &path() const { return path_; }

    bool flush()
    {
        std::FILE *f = std::fopen(path_.c_str(), "wb");
        if (!f) return false;
        bool ok = true;
        for (const auto &kv : vars_) {
            const Var &v = kv.second;
            // MAT level 4 header: type 0000 (little-endian IEEE, fp64, full), rows, cols,
            // imaginary flag, name length incl. NUL; then the name and column-major data
            const int32_t hdr[5] = {0, (int32_t)v.dim, (int32_t)(v.dim ? v.data.size() / v.dim : 0), 0,
                                    (int32_t)kv.first.size() + 1};
            ok = ok && std::fwrite(hdr, sizeof(hdr), 1, f) == 1;
            ok = ok && std::fwrite(kv.first.c_str(), 1, kv.first.size() + 1, f) == kv.first.size() + 1;
            if (!v.data.empty()) ok = ok && std::fwrite(v.data.data(), 8, v.data.size(), f) == v.data.size();
        }
        return std::fclose(f) == 0 && ok;
    }

private:
    struct Var {
        std::size_t dim = 0;
        std::vector<double> data;
    };
    explicit MatLogger(const std::string &prefix) : path_(prefix + ".mat") {}

    bool push(const std::string &name, const double *v, std::size_t dim)
    {
        Var &var = vars_[name];
        if (var.data.empty()) {
            var.dim = dim;
            var.data.reserve(reserve_ * dim);
        }
        if (dim != var.dim) return false; // a variable keeps its dimension
        var.data.insert(var.data.end(), v, v + dim);
        return true;
    }

    std::string path_;
    std::size_t reserve_ = 1024;
    std::map<std::string, Var> vars_;
};

}  // namespace XBot
