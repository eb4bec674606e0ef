"""Test helpers: octrees in the forms the reference's own builders produce.

- writer_encoding(): every octant child re-encoded the way Octant::set_mask_for writes
  ChildType::Octant (new_octree.rs:160-178): bit i+8 set, bit i clear.
- collapse(): leaves above the bottom level, as build_region_octree's LOD / compaction emits
  (RegionSubtreeResult::Lod, new_octree.rs:534-536, 679-690; SectionOctantResult::Lod :599-750):
  chosen octant children are replaced by one leaf whose primitive list is the union of their
  subtree's leaves, so the leaf still holds every primitive that meets its cell.
"""
from __future__ import annotations

import dataclasses

import numpy as np


def writer_encoding(tree):
    """Same octree with every (present, leaf) = (1, 0) octant child stored as (0, 1)."""
    m = tree.octant_mask.astype(np.uint32)
    present, high = m & 0xFF, m >> 8
    octant = present & ~high & 0xFF
    m2 = (present & ~octant) | ((high | octant) << 8)
    return dataclasses.replace(tree, octant_mask=m2.astype(np.uint16))


def _subtree_prims(tree, node, out):
    m = int(tree.octant_mask[node])
    for i in range(8):
        if not (m >> i) & 1:
            continue
        v = int(tree.octant_children[node, i])
        if (m >> (i + 8)) & 1:
            f, c = int(tree.leaf_first[v]), int(tree.leaf_count[v])
            out.update(int(p) for p in tree.leaf_prims[f:f + c])
        else:
            _subtree_prims(tree, v, out)


def _levels(tree):
    """level (distance from the root) of every reachable octant"""
    lv = {tree.root: 0}
    stack = [tree.root]
    while stack:
        n = stack.pop()
        m = int(tree.octant_mask[n])
        for i in range(8):
            if (m >> i) & 1 and not (m >> (i + 8)) & 1:
                c = int(tree.octant_children[n, i])
                lv[c] = lv[n] + 1
                stack.append(c)
    return lv


def collapse(tree, parent_levels, every=2):
    """Collapse every `every`-th octant child of the octants at the given levels (distance from the
    root) into a single leaf.  A child of a level-l octant covers a cell of level depth - 1 - l
    (level 0 = the finest cells), so parent_levels=(0,) puts leaves directly under the root."""
    mask = tree.octant_mask.astype(np.uint32).copy()
    children = tree.octant_children.copy()
    first, count, prims = list(tree.leaf_first), list(tree.leaf_count), list(tree.leaf_prims)
    lv = _levels(tree)
    k = 0
    for node in sorted(lv, key=lambda n: (lv[n], n)):
        if lv[node] not in parent_levels:
            continue
        m = int(mask[node])
        for i in range(8):
            if not (m >> i) & 1 or (m >> (i + 8)) & 1:
                continue
            k += 1
            if k % every:
                continue
            s: set = set()
            _subtree_prims(tree, int(children[node, i]), s)
            lst = sorted(s)
            first.append(len(prims))
            count.append(len(lst))
            prims.extend(lst)
            children[node, i] = len(first) - 1
            mask[node] |= 1 << (i + 8)
    u32 = lambda a: np.asarray(a, np.uint32)  # noqa: E731
    return dataclasses.replace(tree, octant_mask=mask.astype(np.uint16), octant_children=children,
                               leaf_first=u32(first), leaf_count=u32(count), leaf_prims=u32(prims))


def leaf_levels(tree):
    """histogram {cell level: leaf children} of the reachable tree (level 0 = finest cells)"""
    lv = _levels(tree)
    h: dict = {}
    for n, l in lv.items():
        m = int(tree.octant_mask[n])
        for i in range(8):
            if (m >> i) & 1 and (m >> (i + 8)) & 1:
                cl = tree.depth - 1 - l
                h[cl] = h.get(cl, 0) + 1
    return h


def with_octree(scene, tree):
    return dataclasses.replace(scene, octree=tree)
