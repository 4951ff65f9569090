// abi_copy.h -- element-wise copy of an Eigen-style matrix into the row-major layout of the
// C ABI (include/wbq.h). Eigen's MatrixXd is column-major, so data() is never copied as is.
#pragma once

#include <XCM/XBotControlPlugin.h>

inline void copy_row_major(const Eigen::MatrixXd &A, int rows, int cols, double *dst)
{
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) dst[(size_t)r * cols + c] = A(r, c);
}
