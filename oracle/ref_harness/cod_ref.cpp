// cod_ref.cpp -- TEST INFRASTRUCTURE ONLY.  Solves least-squares systems with the reference's own vendored Eigen
// (/root/reference/src/Eigen, compiled where it lies) exactly as renderROMIS does:
//   inline Eigen::VectorXf solveSystem(const Eigen::MatrixXf& A, const Eigen::VectorXf& b)
//   { return A.completeOrthogonalDecomposition().solve(b); }                       (src/rendering/render_utils.h:52)
// stdin : records of  uint32 n, float A[n*n] (column-major), float b[n]   (little-endian binary, until EOF)
// stdout: per record  uint32 rank, float x[n]
// Used once in the build container by tests/golden/make_cod_fixtures.py; its output is committed as fixtures.
#include <Eigen/Dense>

#include <cstdint>
#include <cstdio>

int main() {
    uint32_t n;
    while (std::fread(&n, 4, 1, stdin) == 1) {
        if (n == 0 || n > 64) return 2;
        Eigen::MatrixXf A(n, n);
        Eigen::VectorXf b(n);
        if (std::fread(A.data(), 4, (size_t)n * n, stdin) != (size_t)n * n) return 3;
        if (std::fread(b.data(), 4, n, stdin) != n) return 4;
        Eigen::CompleteOrthogonalDecomposition<Eigen::MatrixXf> cod = A.completeOrthogonalDecomposition();
        Eigen::VectorXf x = cod.solve(b);
        uint32_t rank = (uint32_t)cod.rank();
        std::fwrite(&rank, 4, 1, stdout);
        std::fwrite(x.data(), 4, n, stdout);
    }
    return 0;
}
