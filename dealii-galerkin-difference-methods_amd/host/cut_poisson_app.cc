// cut_poisson_app -- prototypes/cut_poisson_01_gdm.cc over the C ABI: the 2D
// cut Poisson problem (GDM p = 3, 64 x 64 cells on [-1.21, 1.21]^2, unit
// circle, Nitsche, test<2>(false) then test<2>(true) with ghost penalty),
// assembled by libgdm_hip.so, solved by the device SolverCG (identity,
// ReductionControl(n, 1e-10, 1e-6)), the error table printed like the
// reference's ConvergenceTable::write_text (cut_poisson_01_gdm.cc:407-414).
//
//   cut_poisson_app [N_SUB] [DEVICE]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gdm_hip.h"

static void check(int rc, const char *what) {
  if (rc != GDM_OK) {
    char msg[512];
    gdm_last_error(msg, sizeof(msg));
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, msg);
    std::exit(1);
  }
}

static void test(bool ghost_penalty, int n_sub, int device) {
  const double center[2] = {0.0, 0.0};
  gdm_cut_system *S = nullptr;
  check(gdm_cut_poisson_create(3, n_sub, -1.21, 1.21, center, 1.0, ghost_penalty ? 1 : 0, 4.0, 1.0, &S),
        "gdm_cut_poisson_create");
  int64_t n, nnz, n_in, n_cut;
  check(gdm_cut_poisson_info(S, &n, &nnz, &n_in, &n_cut), "gdm_cut_poisson_info");
  gdm_csr *A = nullptr;
  check(gdm_cut_poisson_matrix(S, device, &A), "gdm_cut_poisson_matrix");
  std::vector<double> u((size_t)n);
  int its = 0;
  double res = 0.0;
  check(gdm_cut_poisson_solve(S, A, 1e-6, 1e-10, (int)n, u.data(), &its, &res), "gdm_cut_poisson_solve");
  double err = 0.0;
  check(gdm_cut_poisson_l2_error(S, u.data(), &err), "gdm_cut_poisson_l2_error");
  std::fprintf(stderr, "[cut_poisson_app] gp=%d dofs=%lld nnz=%lld inside=%lld intersected=%lld cg=%d res=%.3e\n",
               ghost_penalty ? 1 : 0, (long long)n, (long long)nnz, (long long)n_in, (long long)n_cut, its, res);
  // ConvergenceTable::write_text: "Mesh size" (default precision 4) and
  // "L2-Error" (scientific, precision 4)
  std::printf("\nMesh size  L2-Error  \n");
  std::printf("   %.4f %.4e \n\n", 2.42 / n_sub, err);
  gdm_csr_destroy(A);
  gdm_cut_poisson_destroy(S);
}

int main(int argc, char **argv) {
  const int n_sub = argc > 1 ? std::atoi(argv[1]) : 64;
  const int device = argc > 2 ? std::atoi(argv[2]) : 0;
  test(false, n_sub, device);
  test(true, n_sub, device);
  return 0;
}
