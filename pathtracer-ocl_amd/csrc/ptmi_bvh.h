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

// Build the index of the triangles below reference node `root` (its subtree in
// `nodes`, triangle ranges tri_off/tri_cnt) into `out`; *entry receives the
// root record (entry code + widened hull).  Returns PTMI_OK or an error.
int build_root_index(const uint8_t* tris, const std::vector<DevNode>& nodes, const std::vector<int32_t>& tri_off,
                     const std::vector<int32_t>& tri_cnt, int32_t root, RootIndex& out, RootRec* rec, char* err,
                     size_t err_len);

}  // namespace ptmi
