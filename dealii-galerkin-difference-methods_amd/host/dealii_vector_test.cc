// dealii_vector_test.cc -- gdm/hip/dealii_vector.h against a stand-in with the
// member names of deal.II's LinearAlgebra::distributed::Vector (owned entries
// followed by ghosts): the owned block lands at the engine-local owned offset
// on every rank of a z-slab partition and comes back unchanged with the ghosts
// zeroed; block(0) goes through the reference <-> device point permutation
// both ways.  Usage: dealii_vector_test [DEVICE]; prints "ok" or fails.
#include <gdm/hip/dealii_vector.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

struct StandInVector {  // LinearAlgebra::distributed::Vector<double>: [owned | ghosts]
  std::vector<double> v;
  std::size_t owned = 0;
  StandInVector(std::size_t n_owned, std::size_t n_ghosts) : v(n_owned + n_ghosts, 0.0), owned(n_owned) {}
  std::size_t locally_owned_size() const { return owned; }
  double *begin() { return v.data(); }
  const double *begin() const { return v.data(); }
  void zero_out_ghost_values() {
    for (std::size_t i = owned; i < v.size(); ++i) v[i] = 0.0;
  }
};

struct StandInBlockVector {
  StandInVector b0, b1;
  StandInVector &block(unsigned int i) { return i == 0 ? b0 : b1; }
  const StandInVector &block(unsigned int i) const { return i == 0 ? b0 : b1; }
};

void require(bool c, const char *what) {
  if (!c) {
    std::fprintf(stderr, "dealii_vector_test: %s\n", what);
    std::exit(1);
  }
}

}  // namespace

int main(int argc, char **argv) {
  const int device = argc > 1 ? std::atoi(argv[1]) : 0;
  using namespace GDM::HIP;
  for (int rank = 0; rank < 3; ++rank) {
    gdm_mesh_desc m{};
    m.dim = 3;
    m.fe_degree = 5;
    m.n_subdivisions[0] = 20;
    m.n_subdivisions[1] = 18;
    m.n_subdivisions[2] = 40;
    for (int d = 0; d < 3; ++d) m.hi[d] = 1.0;
    m.n_ranks = 3;
    m.rank = rank;
    const double a[3] = {0.7, -0.4, 0.3};
    gdm_op *op = nullptr;
    check(gdm_op_create(&m, GDM_OP_ADVECTION, a, 3, device, &op), "gdm_op_create");
    {
      EngineBlockVector eng(op);
      const gdm_layout &L = eng.layout();
      require(owned_offset(L) == (int64_t)L.ghost_planes_below * L.plane_size, "owned offset");
      StandInBlockVector in{StandInVector((std::size_t)L.n_bc_points_ref, 7), StandInVector((std::size_t)L.n_owned, 13)};
      for (std::size_t i = 0; i < in.b1.v.size(); ++i) in.b1.v[i] = std::sin(0.001 * (double)i + rank);
      for (std::size_t i = 0; i < in.b0.v.size(); ++i) in.b0.v[i] = std::cos(0.01 * (double)i - rank);
      eng.import(in);
      // the engine-local buffer: owned block at owned_offset, device block(0) in device order
      const std::vector<double> local = eng.block(1).download();
      for (int64_t i = 0; i < L.n_owned; ++i) require(local[(size_t)(owned_offset(L) + i)] == in.b1.v[(size_t)i], "owned block");
      std::vector<int64_t> ref_to_dev((std::size_t)L.n_bc_points_ref);
      if (L.n_bc_points_ref) check(gdm_bc_reference_order(op, ref_to_dev.data()), "gdm_bc_reference_order");
      const std::vector<double> dev0 = eng.block(0).download();
      for (std::size_t i = 0; i < ref_to_dev.size(); ++i) require(dev0[(size_t)ref_to_dev[i]] == in.b0.v[i], "block(0) order");
      StandInBlockVector out{StandInVector((std::size_t)L.n_bc_points_ref, 7), StandInVector((std::size_t)L.n_owned, 13)};
      for (double &x : out.b1.v) x = -1.0;
      for (double &x : out.b0.v) x = -1.0;
      eng.export_to(out);
      for (int64_t i = 0; i < L.n_owned; ++i) require(out.b1.v[(size_t)i] == in.b1.v[(size_t)i], "round trip (owned)");
      for (std::size_t i = (std::size_t)L.n_owned; i < out.b1.v.size(); ++i) require(out.b1.v[i] == 0.0, "ghosts zeroed");
      for (std::size_t i = 0; i < ref_to_dev.size(); ++i) require(out.b0.v[i] == in.b0.v[i], "round trip (block 0)");
      bool threw = false;
      try {
        StandInBlockVector bad{StandInVector(1, 0), StandInVector((std::size_t)L.n_owned + 1, 0)};
        eng.import(bad);
      } catch (const Error &) {
        threw = true;
      }
      require(threw, "a vector of another slab must be refused");
    }
    gdm_op_destroy(op);
  }
  std::printf("dealii_vector_test ok\n");
  return 0;
}
