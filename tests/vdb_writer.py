"""Minimal OpenVDB (file version 224) writer for loader tests (test
infrastructure only).

Writes a float 'density' grid and a vec3s 'albedo' grid, each a root node
with one 32^3-internal child holding 16^3-internal children, 8^3 leaves and
optional active tiles, in the layout io::File/RootNode/InternalNode/LeafNode
read (tree/RootNode.h readTopology, InternalNode.h readTopology,
LeafNode.h readBuffers, io/Compression.h readCompressedValues).

    nodes = {"leaves": [((ox, oy, oz), mask_bool[512], values[512 x C])],
             "tiles16": [((ox, oy, oz), value)],   # active 8^3 tiles in a 16^3 node
             "tiles32": [((ox, oy, oz), value)]}   # active 128^3 tiles in the 32^3 node
    write_vdb(path, {"density": (nodes, 1), "albedo": (nodes3, 3)}, mode)

mode: "raw" (no compression, all values), "zip" (zlib streams + active-mask
compression), "mask1" (active-mask compression with one stored inactive value,
raw streams), "blosc_memcpy" (blosc frames stored uncompressed).
"""
import struct
import zlib

import numpy as np

COMPRESS_ZIP, COMPRESS_ACTIVE_MASK, COMPRESS_BLOSC = 1, 2, 4


def _str(s):
    b = s.encode()
    return struct.pack("<I", len(b)) + b


def _mask(bits):
    bits = np.asarray(bits, bool)
    words = np.zeros((len(bits) + 63) // 64, np.uint64)
    for i in np.nonzero(bits)[0]:
        words[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
    return words.tobytes()


def _stream(data, flags):
    if flags & COMPRESS_ZIP:
        z = zlib.compress(data)
        return struct.pack("<q", len(z)) + z
    if flags & COMPRESS_BLOSC:  # blosc frame with the whole buffer stored raw (flag 0x02)
        frame = struct.pack("<BBBBIII", 2, 1, 0x02 | 0x20, 4, len(data), len(data), 16 + len(data)) + data
        return struct.pack("<q", len(frame)) + frame
    return data


def _values(vals, active, flags, mode, channels):
    """readCompressedValues: metadata byte, optional inactive value(s) and
    selection mask, then the (active) values."""
    vals = np.asarray(vals, np.float32).reshape(len(active), channels)
    if mode == "mask1":
        inactive = vals[~active][0] if (~active).any() else np.zeros(channels, np.float32)
        return (struct.pack("<b", 4) + inactive.astype(np.float32).tobytes() + _mask(np.zeros(len(active), bool))
                + _stream(vals[active].tobytes(), flags))
    if flags & COMPRESS_ACTIVE_MASK and not active.all():
        return struct.pack("<b", 3) + _mask(np.zeros(len(active), bool)) + _stream(vals[active].tobytes(), flags)
    return struct.pack("<b", 6) + _stream(vals.tobytes(), flags)


def _grid(nodes, channels, flags, mode):
    bg = np.zeros(channels, np.float32)
    out = struct.pack("<I", flags) + struct.pack("<i", 0)      # compression, no grid metadata
    out += _str("UniformScaleMap") + bytes(5 * 24)             # transform
    out += struct.pack("<i", 1) + bg.tobytes() + struct.pack("<II", 0, 1)  # 1 buffer, 0 tiles, 1 child
    out += struct.pack("<iii", 0, 0, 0)                         # 32^3 node at the origin
    # 32^3 node: children = 16^3 nodes holding the leaves / 8^3 tiles
    kids16 = {}
    for (o, m, v) in nodes.get("leaves", []):
        kids16.setdefault(tuple(c // 128 * 128 for c in o), []).append(("leaf", o, m, v))
    for (o, val) in nodes.get("tiles16", []):
        kids16.setdefault(tuple(c // 128 * 128 for c in o), []).append(("tile", o, None, val))
    cm32 = np.zeros(32 ** 3, bool)
    vm32 = np.zeros(32 ** 3, bool)
    v32 = np.zeros((32 ** 3, channels), np.float32)
    for o in kids16:
        cm32[(o[0] // 128) * 1024 + (o[1] // 128) * 32 + o[2] // 128] = True
    for (o, val) in nodes.get("tiles32", []):
        i = (o[0] // 128) * 1024 + (o[1] // 128) * 32 + o[2] // 128
        vm32[i] = True
        v32[i] = val
    out += _mask(cm32) + _mask(vm32) + _values(v32, vm32, flags, mode, channels)
    leaves_in_order = []
    for i in np.nonzero(cm32)[0]:
        o16 = (int(i // 1024) * 128, int(i // 32 % 32) * 128, int(i % 32) * 128)
        items = kids16[o16]
        cm = np.zeros(4096, bool)
        vm = np.zeros(4096, bool)
        vv = np.zeros((4096, channels), np.float32)
        leafs = {}
        for (kind, o, m, v) in items:
            j = ((o[0] - o16[0]) // 8) * 256 + ((o[1] - o16[1]) // 8) * 16 + (o[2] - o16[2]) // 8
            if kind == "leaf":
                cm[j] = True
                leafs[j] = (m, v)
            else:
                vm[j] = True
                vv[j] = v
        out += _mask(cm) + _mask(vm) + _values(vv, vm, flags, mode, channels)
        for j in np.nonzero(cm)[0]:
            m, v = leafs[j]
            out += _mask(m)
            leaves_in_order.append((m, v))
    for (m, v) in leaves_in_order:  # buffers
        out += _mask(m) + _values(v, np.asarray(m, bool), flags, mode, channels)
    return out


def write_vdb(path, grids, mode="raw"):
    flags = {"raw": 0, "zip": COMPRESS_ZIP | COMPRESS_ACTIVE_MASK, "mask1": COMPRESS_ACTIVE_MASK,
             "blosc_memcpy": COMPRESS_BLOSC | COMPRESS_ACTIVE_MASK}[mode]
    head = struct.pack("<qIIIB", 0x56444220, 224, 8, 1, 1) + b"0" * 36 + struct.pack("<i", 0)
    head += struct.pack("<i", len(grids))
    body = head
    for name, (nodes, channels) in grids.items():
        typ = "Tree_float_5_4_3" if channels == 1 else "Tree_vec3s_5_4_3"
        desc_len = len(_str(name)) + len(_str(typ)) + len(_str("")) + 24
        grid = _grid(nodes, channels, flags, mode)
        gpos = len(body) + desc_len
        body += _str(name) + _str(typ) + _str("") + struct.pack("<qqq", gpos, gpos, gpos + len(grid)) + grid
    with open(path, "wb") as f:
        f.write(body)
