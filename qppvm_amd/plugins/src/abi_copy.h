// abi_copy.h -- element-wise copies of Eigen / KDL values into the row-major layouts of the C
// ABI (include/wbq.h). Eigen's MatrixXd is column-major, so data() is never copied as is.
#pragma once

#include <XCM/XBotControlPlugin.h>

inline void copy_row_major(const Eigen::MatrixXd &A, int rows, int cols, double *dst)
{
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) dst[(size_t)r * cols + c] = A(r, c);
}

// pose [R | p] as 3x4 row-major (the top three rows of Affine3d::matrix())
inline void copy_pose(const Eigen::Affine3d &T, double *dst)
{
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) dst[4 * r + c] = T.linear()(r, c);
        dst[4 * r + 3] = T.translation()(r);
    }
}

inline void copy_pose(const KDL::Frame &F, double *dst)
{
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) dst[4 * r + c] = F.M(r, c);
        dst[4 * r + 3] = F.p(r);
    }
}
