// ptmi_bvh.h -- host builder of the per-root triangle traversal index (ptmi_bvh.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "ptmi_device.h"

namespace ptmi {

struct RootIndex {  // appended to by every root built into one scene
    std::vector<Node4> nodes;
    std::vector<DevTri> tris;
    std::vector<ChainBox> chain_boxes;
};

// Build the traversal index of all triangles below the reference roots
// roots[0..n_roots) of one group object (their subtrees in `nodes`, triangle
// ranges tri_off/tri_cnt) into `out`; *rec receives the entry code and the
// widened hull.  Each triangle's gate chain starts with the object's own box
// gate_mn/gate_mx (group space).  Returns PTMI_OK or an error.
int build_object_index(const uint8_t* tris, const std::vector<DevNode>& nodes, const std::vector<int32_t>& tri_off,
                       const std::vector<int32_t>& tri_cnt, const int32_t* roots, int n_roots, const double* gate_mn,
                       const double* gate_mx, RootIndex& out, RootRec* rec, char* err, size_t err_len);

// After every object of a scene is built into `idx` (codes in the builder's wide format):
// appends the sentinel triangle of the empty slots and re-codes every Node4 child and root
// entry in the scene's final format (ptmi_device.h Node4).  Returns the leaf bit:
// kLeafNarrow when every code fits 16 bits, else kLeafWide.
int32_t finalize_index_codes(RootIndex& idx, std::vector<RootRec>& recs);

}  // namespace ptmi
