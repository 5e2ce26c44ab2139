// gdm/hip/dealii_vector.h -- the adapter between deal.II's distributed vectors
// and the engine's device buffers (what INTEGRATION.md §2 calls the
// EngineBlockVector): header-only, templated on the vector types so it carries
// no deal.II dependency (none is in this image).  It relies on this part of the
// LinearAlgebra::distributed::Vector<double, MemorySpace::Host> interface:
//
//   locally_owned_size()     owned entries of this rank (deal.II >= 9.3)
//   begin()                  pointer to the owned entries (ghosts follow them)
//   zero_out_ghost_values()  ghost entries invalidated after an owned write
//
// and, for the advection BlockVector (problem.h:62-76), block(0) / block(1).
//
// Layouts.  The reference orders a rank's owned DoFs lexicographically inside
// its z-slab (system.h:238-244); the engine's local buffer is
// [p ghost planes | owned planes | p ghost planes] of the same order
// (gdm_layout), so the owned block maps one to one at owned_offset.  deal.II's
// ghosts (one ghost cell layer) are not the p planes the owner-computes stencil
// reads: they come from the engine's exchange (Communicator), never from here.
// block(0) (stage boundary values) is in the reference's point_counter order
// over the owned cells (stiffness.h:40-160); the engine's block(0) is in face
// order and also holds the neighbour cells' points (owner-computes), so values
// are scattered through gdm_bc_reference_order and the extra points are the
// caller's to fill (gdm_eval_boundary on the device, or host values at
// gdm_bc_points).
#pragma once

#include <gdm/hip/operators.h>

#include <cstdint>
#include <vector>

namespace GDM {
namespace HIP {

// first owned entry of the engine-local buffer (after the ghost planes below)
inline int64_t owned_offset(const gdm_layout &L) { return (int64_t)L.ghost_planes_below * L.plane_size; }

// owned block of a deal.II vector -> the engine-local device buffer
template <typename VectorType>
void copy_owned_to_engine(const VectorType &src, gdm_op *op, const gdm_layout &L, DeviceVector &local) {
  if ((int64_t)src.locally_owned_size() != L.n_owned || (int64_t)local.size() != L.n_local)
    throw Error("copy_owned_to_engine: the vector's owned range is not the operator's slab");
  if (L.n_owned)
    check(gdm_memcpy_h2d(op, local.get_values() + owned_offset(L), &*src.begin(), sizeof(double) * L.n_owned),
          "gdm_memcpy_h2d");
}

// engine-local device buffer -> owned block of a deal.II vector (ghosts zeroed:
// they are stale until the caller's next update_ghost_values)
template <typename VectorType>
void copy_owned_from_engine(const DeviceVector &local, gdm_op *op, const gdm_layout &L, VectorType &dst) {
  if ((int64_t)dst.locally_owned_size() != L.n_owned || (int64_t)local.size() != L.n_local)
    throw Error("copy_owned_from_engine: the vector's owned range is not the operator's slab");
  if (L.n_owned)
    check(gdm_memcpy_d2h(op, &*dst.begin(), local.get_values() + owned_offset(L), sizeof(double) * L.n_owned),
          "gdm_memcpy_d2h");
  dst.zero_out_ghost_values();
}

// The advection BlockVector's two blocks on the device: block(0) = stage
// boundary values (engine order), block(1) = DoF values (engine-local layout);
// moves to and from a deal.II BlockVector (block(0) in the reference order).
class EngineBlockVector : public BlockVector {
 public:
  EngineBlockVector(gdm_op *op) : op_(op) {
    check(gdm_op_layout(op_, &layout_), "gdm_op_layout");
    b0.reinit(op_, (std::size_t)std::max<int64_t>(layout_.n_bc_points, 1));
    b1.reinit(op_, (std::size_t)layout_.n_local);
    ref_to_dev_.resize((std::size_t)layout_.n_bc_points_ref);
    if (layout_.n_bc_points_ref)
      check(gdm_bc_reference_order(op_, ref_to_dev_.data()), "gdm_bc_reference_order");
  }

  template <typename BlockVectorType>
  void import(const BlockVectorType &src) {
    copy_owned_to_engine(src.block(1), op_, layout_, b1);
    if ((int64_t)src.block(0).locally_owned_size() != layout_.n_bc_points_ref)
      throw Error("EngineBlockVector::import: block(0) is not the reference's boundary-point block");
    std::vector<double> dev((std::size_t)std::max<int64_t>(layout_.n_bc_points, 1), 0.0);
    const double *ref = &*src.block(0).begin();
    for (std::size_t i = 0; i < ref_to_dev_.size(); ++i) dev[(std::size_t)ref_to_dev_[i]] = ref[i];
    b0.upload(dev);
  }

  template <typename BlockVectorType>
  void export_to(BlockVectorType &dst) const {
    copy_owned_from_engine(b1, op_, layout_, dst.block(1));
    if ((int64_t)dst.block(0).locally_owned_size() != layout_.n_bc_points_ref)
      throw Error("EngineBlockVector::export_to: block(0) is not the reference's boundary-point block");
    const std::vector<double> dev = b0.download();
    double *ref = &*dst.block(0).begin();
    for (std::size_t i = 0; i < ref_to_dev_.size(); ++i) ref[i] = dev[(std::size_t)ref_to_dev_[i]];
    dst.block(0).zero_out_ghost_values();
  }

  const gdm_layout &layout() const { return layout_; }

 private:
  gdm_op *op_;
  gdm_layout layout_{};
  std::vector<int64_t> ref_to_dev_;
};

}  // namespace HIP
}  // namespace GDM
