"""Test infrastructure: the reference's section octree builder restated in Python, and an independent
voxel DDA for block-value scenes.

section_octants() builds a 16^3 block array the way SectionOctantBuilder::section_data_to_octants
(src/octree/new_octree.rs:599-710, called by section_to_compacted_octree :712-750) is meant to:

- the blocks in Morton order (encode_morton, :752-755; 0 = air = no child, NonZeroU32, :744);
- every group of eight siblings becomes an octant, or -- when Octant::is_compactable holds (:227-233:
  all eight leaf bits set and every child value equal to children[1], or no child at all) -- one leaf
  holding that value (or nothing) of its parent (leaves_to_child :664-686, insert_child_and_compact
  :688-709), bottom-up to the section root (:632-640: a compactable root is SectionOctantResult::Lod or
  Empty);
- octants are pushed as they complete (children before parents), the root last; the list is then
  reversed and child ids renumbered `len - id`, so the root is octant 0 (:641-661);
- masks in the writer's encoding: a leaf child sets bits i and i + 8, an octant child bit i + 8 alone
  (Octant::set_mask_for :160-178).

As written the streaming builder does not produce that tree: Octant::free_slot (:260-270)
looks for the lowest clear bit of the whole 16-bit mask, and neither an empty child nor an octant child
(bit i + 8 alone) sets bit i, so such children do not occupy their slot; the carry of a full buffer
(:695-706) replaces the child being inserted, which is lost; and the last buffers are never carried into
the root.  section_octants restates the algorithm those lines implement in intent; the defects are not
replicated.
"""
from __future__ import annotations

import numpy as np

SECTION = 16


def encode_morton(x: int, y: int, z: int) -> int:
    """new_octree.rs:752-755 (part_by_2 :813-822): x bit 0, y bit 1, z bit 2."""
    code = 0
    for b in range(21):
        code |= ((x >> b) & 1) << (3 * b) | ((y >> b) & 1) << (3 * b + 1) | ((z >> b) & 1) << (3 * b + 2)
    return code


def _is_compactable(mask: int, children: list) -> bool:
    """Octant::is_compactable (new_octree.rs:227-233)."""
    first = children[1]
    return (((mask >> 8) & 0xFF) == 0xFF and all(c == first for c in children)) or mask == 0


def section_octants(grid: np.ndarray):
    """grid[x, y, z] (16^3 uint32, 0 = air) -> ("subtree", masks uint16[n], children uint32[n, 8]) with
    the root at 0, or ("lod", value) / ("empty", 0) -- SectionOctantResult (new_octree.rs:605-614)."""
    assert grid.shape == (SECTION,) * 3
    data = [0] * (SECTION ** 3)
    for x in range(SECTION):
        for y in range(SECTION):
            for z in range(SECTION):
                data[encode_morton(x, y, z)] = int(grid[x, y, z])
    pushed = []  # (mask, children) in completion order

    def node(lo: int, size: int):
        """(kind, value) of the child covering Morton codes [lo, lo + size): 'empty' / 'leaf' / 'octant'."""
        mask, ch = 0, [0] * 8
        step = size // 8
        for i in range(8):
            if step == 1:
                v = data[lo + i]
                kind, val = ("leaf", v) if v else ("empty", 0)
            else:
                kind, val = node(lo + i * step, step)
            if kind == "leaf":
                mask |= (1 << i) | (1 << (i + 8))
            elif kind == "octant":
                mask |= 1 << (i + 8)  # set_mask_for(ChildType::Octant): bit i + 8 alone
            ch[i] = val
        if _is_compactable(mask, ch):
            return ("leaf", ch[0]) if mask else ("empty", 0)
        pushed.append((mask, ch))
        return "octant", len(pushed) - 1

    # the section root (:632-640) is compacted like any octant, but reported as Lod / Empty
    kind, val = node(0, SECTION ** 3)
    if kind == "leaf":
        return "lod", val
    if kind == "empty":
        return "empty", 0
    n = len(pushed) - 1  # octants_len before the root's push (:641)
    masks = np.zeros(len(pushed), np.uint16)
    children = np.zeros((len(pushed), 8), np.uint32)
    for j, (mask, ch) in enumerate(pushed):
        out = n - j  # self.octants.reverse() (:656): original j lands at n - j
        masks[out] = mask
        for i in range(8):
            is_octant = (mask >> (i + 8)) & 1 and not (mask >> i) & 1
            children[out, i] = (n - ch[i]) if is_octant else ch[i]  # new_id = octants_len - id (:650)
    return "subtree", masks, children


def decode_cell(masks: np.ndarray, children: np.ndarray, root: int, depth: int, x: int, y: int, z: int) -> int:
    """The leaf value the octree holds at cell (x, y, z) (0 = empty), reading either mask encoding (C21)."""
    node = root
    for level in range(depth - 1, -1, -1):
        i = ((x >> level) & 1) | (((y >> level) & 1) << 1) | (((z >> level) & 1) << 2)
        m = int(masks[node])
        present, high = (m >> i) & 1, (m >> (i + 8)) & 1
        if not present and not high:
            return 0
        if present and high:
            return int(children[node, i])
        node = int(children[node, i])
    raise AssertionError("descended below the leaf level")


def dda_first_block(grid: np.ndarray, origin, direction, opaque=None):
    """Independent check (Amanatides & Woo voxel walk in float64) of the first non-air cell a ray enters
    from outside the grid: (block, axis, t) or None.  grid[x, y, z], cell k spans [k, k + 1)."""
    n = np.array(grid.shape, np.int64)
    o = np.asarray(origin, np.float64)
    d = np.asarray(direction, np.float64)
    inv = np.where(d != 0.0, 1.0 / np.where(d != 0.0, d, 1.0), np.inf)
    t0 = np.where(d != 0.0, (np.where(d > 0, 0.0, n) - o) * inv, -np.inf)
    t1 = np.where(d != 0.0, (np.where(d > 0, n, 0.0) - o) * inv, np.inf)
    for a in range(3):
        if d[a] == 0.0 and not (0.0 <= o[a] < n[a]):
            return None
    t_in, t_out = max(t0.max(), 0.0), t1.min()
    if t_in >= t_out:
        return None
    axis = int(np.argmax(t0)) if t0.max() > 0 else -1
    p = o + d * t_in
    cell = np.clip(np.floor(p).astype(np.int64), 0, n - 1)
    if axis >= 0:  # entering through a face: the cell just inside it
        cell[axis] = 0 if d[axis] > 0 else n[axis] - 1
    step = np.where(d > 0, 1, -1)
    nxt = np.where(d > 0, cell + 1, cell).astype(np.float64)
    t_next = np.where(d != 0.0, (nxt - o) * inv, np.inf)
    t = t_in
    while True:
        v = int(grid[tuple(cell)])
        if v and (opaque is None or opaque(v)):
            return v, axis, t
        a = int(np.argmin(t_next))
        t = t_next[a]
        if t >= t_out:
            return None
        cell[a] += step[a]
        if not (0 <= cell[a] < n[a]):
            return None
        t_next[a] += abs(inv[a])
        axis = a
