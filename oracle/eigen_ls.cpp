// oracle/eigen_ls.cpp -- TEST INFRASTRUCTURE (oracle/_ref only; never linked into the product).
//
// The 3x3 linear solver of BCM's Eigen SUNLinearSolver (src/odecommon/sunlinsol_dense_eigen.cpp:
// 130-143 setup, 169-176 solve) evaluated by the reference's own vendored Eigen
// (dependencies/eigen-3.4-rc1, included where it lies by oracle/Makefile): the cofactor inverse
// Eigen::internal::compute_inverse<MatrixXd, Matrix3d, 3>::run into a Matrix3d, then
// x.noalias() = inverse * b. backend_ref.c calls these for N = 3, so the bit-for-bit comparison of
// the restatement with _ref/libbcm3ref_nofma.so (tests/test_oracle.py) also pins the restated
// inverse (backend_restated.c, and the device's closed-form inverse) to Eigen's arithmetic.
#include <Eigen/Dense>

extern "C" {

// a: the SUNDenseMatrix data (column-major 3 x 3); inv: row-major 3 x 3
void eigenref_inverse3(const double* a, double* inv)
{
    Eigen::MatrixXd A(3, 3);
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) A(i, j) = a[j * 3 + i];
    Eigen::Matrix3d R;
    Eigen::internal::compute_inverse<Eigen::MatrixXd, Eigen::Matrix3d, 3>::run(A, R);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) inv[i * 3 + j] = R(i, j);
}

void eigenref_solve3(const double* inv, const double* b, double* x)
{
    Eigen::Matrix3d R;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R(i, j) = inv[i * 3 + j];
    Eigen::VectorXd bv(3), xv(3);
    for (int i = 0; i < 3; i++) bv(i) = b[i];
    xv.noalias() = R * bv;
    for (int i = 0; i < 3; i++) x[i] = xv(i);
}

}  // extern "C"
