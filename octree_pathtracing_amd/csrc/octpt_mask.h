// octpt_mask.h -- the octant child encodings the boundary accepts.
//
// new_octree::Octant keeps two bits per child i in its u16 child_mask.  The reference reads
// them as "bit i = present, bit i+8 = leaf" (OctantChildIterator, new_octree.rs:84-100;
// is_child / is_leaf :144-156), but its only writer, Octant::set_mask_for (:160-178), encodes
// ChildType::Octant as bit i+8 set and bit i CLEAR -- the form every tree built by
// expand_by / RegionOctreeBuilder / SectionOctantBuilder carries (:60, 541, 566, 684, 703).
// The four combinations are distinct, so the upload accepts both writers' octants:
//   (bit i, bit i+8) = (0,0) empty, (1,0) octant (reader form), (0,1) octant (set_mask_for
//   form), (1,1) leaf.
// normalized_mask() maps a mask to the reader form, which is what the device layout and the
// traversals consume.
#pragma once
#include <stdint.h>

namespace octpt {

inline uint16_t normalized_mask(uint16_t m) {
    const uint32_t present = m & 0xFFu, high = (uint32_t)m >> 8;
    const uint32_t leaf = present & high;            // (1,1)
    const uint32_t octant_w = high & ~present;       // (0,1): set_mask_for(ChildType::Octant)
    return (uint16_t)((present | octant_w) | (leaf << 8));
}

}  // namespace octpt
