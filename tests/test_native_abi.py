"""The C ABI: the library loads and exports every symbol include/matcha_gossip.h declares; host-side
entry points and argument validation work without a GPU."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "matcha_gossip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mx_[a-z0-9_]+)\s*\(", txt)))


def test_exports_every_declared_symbol(pkg):
    names = _declared()
    assert len(names) >= 20
    so = ctypes.CDLL(pkg._lib.LIB_PATH)
    for n in names:
        assert hasattr(so, n), n
    assert set(names) == set(pkg._lib.SIGNATURES), "ctypes table out of sync with the header"


def test_version_and_plan_geometry(pkg):
    L = pkg.lib
    assert L.mx_version().startswith(b"matcha-gossip")
    assert L.mx_plan_words(8, 5) == 4 + 2 * 8 + 8 * 5
    assert L.mx_mix_tile(8) == 1024 and L.mx_mix_tile(16) == 1024
    assert L.mx_mix_tile(32) == 512 and L.mx_mix_tile(64) == 256 and L.mx_mix_tile(65) == 256
    assert L.mx_mix_tile(156) == 256 and L.mx_mix_tile(157) == 0          # mix_kernel_wide up to 156 slots
    assert L.mx_choco_msg_bytes(10, 3) == 4 * 4 + 8 * 3 + 4 * 2          # + tile bounds [1 tile + 1]
    assert L.mx_choco_msg_bytes(8193, 4) == 4 * 4 + 8 * 4 + 4 * 4        # 3 tiles of 4096
    assert L.mx_choco_apply_work_bytes(1 << 20, 8) == 0


def test_mix_layout(pkg):
    L = pkg.lib
    lens = np.array([0, 1, 1024, 1025, 5], np.int64)
    off = np.zeros(6, np.int64)
    assert L.mx_mix_layout(lens.ctypes.data, 5, 8, off.ctypes.data) == 0
    assert off.tolist() == [0, 0, 1, 2, 4, 5]


def test_invalid_arguments_report_errors(pkg):
    L = pkg.lib
    rc = L.mx_gossip_mix(None, None, None, None, 1, 1, 8, None, 0, 8, 5, 0.25, None)
    assert rc == -1 and b"null" in L.mx_last_error()
    key = np.zeros(624, np.uint32)
    p = np.array([1.5])
    out = np.zeros(624, np.uint32)
    pos = ctypes.c_int(0)
    rc = L.mx_flags_binomial(key.ctypes.data, 624, p.ctypes.data, 1, 10, ctypes.c_void_p(16),
                             out.ctypes.data, ctypes.byref(pos), None)
    assert rc == -1 and b"> 1" in L.mx_last_error()
    assert L.mx_topk_abs_diff(None, None, 10, 11, None, None, None, None) == -1
    # the pull transport's Choco entries validate before touching a device
    assert L.mx_pull_fetch(None, 1, 2, None, None, 256, 100, None) == -1 and b"null" in L.mx_last_error()
    fake = ctypes.c_void_p(256)
    assert L.mx_pull_fetch(fake, 1, 2, fake, fake, 96, 100, None) == -1 and b"dst_ld" in L.mx_last_error()
    assert L.mx_choco_apply_slots(fake, fake, fake, 8, 8, 1, None, 2, fake, 0, 1, 1, 0.5, 0.1, None) == -1
    assert b"slot table" in L.mx_last_error()


def test_dropin_shims_resolve(pkg):
    import importlib.util
    import sys
    d = os.path.join(ROOT, pkg.__name__, "dropin")
    sys.path.insert(0, d)
    try:
        for mod in ("graph_manager", "communicator", "comm_helpers", "compressors"):
            spec = importlib.util.spec_from_file_location("dropin_" + mod, os.path.join(d, mod + ".py"))
            m = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(m)
        assert m.get_top_k is pkg.get_top_k
    finally:
        sys.path.remove(d)


def test_exchange_plan_moves_each_row_once_per_link(pkg):
    """Graph 0 split over 2 GPUs ({0-3}, {4-7}), every matching active: 6 cross edges, but workers
    0 (partners 4, 7), 1 (5, 7) and 3 (6, 7) each cross the link once, and 7 (partners 0, 1, 3)
    once the other way -- 3 rows 0 -> 1 and 4 rows 1 -> 0 instead of 6 + 6 (mx_exchange_plan)."""
    import ctypes
    import numpy as np
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
    partner = np.ascontiguousarray(np.asarray(gp.neighbors_info, np.int32))
    M = partner.shape[0]
    owner = pkg.engine.owner_table(8, 2)
    flags = np.ones(M, np.uint8)
    for rank, (base, nl) in enumerate(pkg.partition(8, 2)):
        cnt = ctypes.c_int(0)
        assert pkg.lib.mx_exchange_plan(flags.ctypes.data, M, partner.ctypes.data, 8, owner.ctypes.data, rank,
                                        base, nl, None, 0, ctypes.byref(cnt)) == 0
        ops = np.zeros((cnt.value, 4), np.int32)
        assert pkg.lib.mx_exchange_plan(flags.ctypes.data, M, partner.ctypes.data, 8, owner.ctypes.data, rank,
                                        base, nl, ops.ctypes.data, cnt.value, ctypes.byref(cnt)) == 0
        sends = sorted(int(o[3]) for o in ops if o[0] == 0)
        recvs = [int(o[3]) for o in ops if o[0] == 1]
        assert len(set(sends)) == len(sends) and len(set(recvs)) == len(recvs)
        assert [int(o[2]) for o in ops if o[0] == 1] == list(range(len(recvs)))    # slab slots
        assert (len(sends), len(recvs)) == ((3, 4) if rank == 0 else (4, 3))
        assert sends == ([0, 1, 3] if rank == 0 else [4, 5, 6, 7])
        assert pkg.engine.max_incoming_remote(partner, base, nl) == len(recvs)


def test_mix_kernel_dispatch_names(pkg):
    """mx_mix_kernel_name mirrors mx_gossip_mix's dispatch under the knobs (host-only)."""
    E = pkg.engine
    saved = E.mix_tuning()
    try:
        assert saved["rows"] == 2
        assert [E.mix_kernel_name(s) for s in (1, 8, 9, 16, 33, 64)] == ["mix_kernel_rows"] * 6
        assert E.mix_kernel_name(65) == E.mix_kernel_name(156) == "mix_kernel_wide"
        assert E.mix_kernel_name(157) == ""
        E.set_mix_tuning(rows=1)
        assert [E.mix_kernel_name(s) for s in (8, 16, 64)] == ["mix_kernel_reg", "mix_kernel_rows", "mix_kernel_rows"]
        E.set_mix_tuning(rows=0, regidx=0)
        assert [E.mix_kernel_name(s) for s in (8, 16)] == ["mix_kernel", "mix_kernel"]
        E.set_mix_tuning(rows=2, regidx=1, unroll=4)
        assert [E.mix_kernel_name(s) for s in (8, 16)] == ["mix_kernel_reg", "mix_kernel_rows"]
        assert pkg.lib.mx_mix_set(b"rows", 3) != 0
    finally:
        E.set_mix_tuning(**saved)


def test_mean_rows_to_refuses_partial_overlap_and_names_kernels(pkg):
    """a destination overlapping the rows at a column offset is refused before any
    launch (host-side validation, fake device addresses); whole-row aliasing passes validation.
    mx_mean_kernel_name follows the launch dispatch (the bench's centralized figure)."""
    L = pkg.lib
    base, ld, count = 1 << 40, 1024, 1000
    rc = L.mx_mean_rows_to(base, 8, ld, count, 0, base + 4 * 16, 8, ld, None)   # 16 columns in
    assert rc == -1 and b"column offset" in L.mx_last_error()
    rc = L.mx_mean_rows_to(base, 8, ld, count, 0, base + 4 * (3 * ld + 5), 1, count, None)
    assert rc == -1 and b"column offset" in L.mx_last_error()
    A = 1 << 40                                       # 16-byte aligned fake addresses (nothing launched)

    def name(nrows, count, order, ld=None, base=A, dst_ld=None):
        ld = ld if ld is not None else (count + 63) // 64 * 64
        return L.mx_mean_kernel_name(base, nrows, ld, count, order, base, nrows, dst_ld if dst_ld else ld)
    assert name(8, 25_600_000, 0) == b"mean_tile_kernel<1>"
    assert name(8, 25_600_000, 1) == b"mean_tile_kernel<0>"
    assert name(8, 400, 0) == b"mean4_kernel<1, 4>"
    assert name(16, 4096, 1) == b"mean4_kernel<0, 4>"
    assert name(16, 4096, 0) == b"mean_to_kernel<float, 1, 64>"
    assert name(65, 4096, 0) == b"mean_to_kernel<float, 2, 1>"
    # the dispatch's alignment conditions -- unaligned rows / ld / dst_ld take the scalar path
    assert name(8, 25_600_000, 0, base=A + 4) == b"mean_to_kernel<float, 1, 8>"
    assert name(8, 25_600_000, 1, ld=25_600_002) == b"mean_to_kernel<float, 0, 1>"
    assert name(8, 25_600_000, 0, dst_ld=25_600_006) == b"mean_to_kernel<float, 1, 8>"
    assert name(8, 100, 0, ld=50) == b"invalid"


def test_ipc_knobs_and_publish_rows_validation(pkg):
    """mx_ipc_set / mx_ipc_get (the export probe's knobs, include/matcha_gossip.h) and the host-side
    argument checks of mx_snapshot_publish_rows (no launch: fake device addresses)."""
    import ctypes
    L = pkg.lib
    g0 = L.mx_ipc_get(b"granule")
    assert g0 == 2 << 20 and L.mx_ipc_get(b"tries") == -1 and L.mx_ipc_get(b"nope") == -1
    try:
        assert L.mx_ipc_set(b"granule", 1) == 0 and L.mx_ipc_get(b"granule") == 1
        assert L.mx_ipc_set(b"granule", 0) != 0 and L.mx_ipc_set(b"tries", 2) != 0
        assert L.mx_ipc_set(b"nope", 1) != 0 and b"unknown" in L.mx_last_error()
    finally:
        L.mx_ipc_set(b"granule", g0)
    ex, ref = ctypes.c_int(-1), ctypes.c_int(-1)
    assert L.mx_ipc_stats(ctypes.byref(ex), ctypes.byref(ref)) == 0 and ex.value >= 0 and ref.value >= 0
    fake = 1 << 40
    assert L.mx_snapshot_publish_rows(fake, 8, fake, 8, 6, 2, fake, 5, fake, 8, 0, None) != 0      # n % 4
    assert L.mx_snapshot_publish_rows(fake, 8, fake, 8, 8, 2, fake, 5, fake, 8, 7, None) != 0      # block
    assert L.mx_snapshot_publish_rows(None, 8, fake, 8, 8, 2, fake, 5, fake, 8, 0, None) != 0      # null
    assert L.mx_snapshot_publish_rows(fake, 8, fake, 8, 0, 2, fake, 5, fake, 8, 0, None) == 0      # nothing to do


def test_mix_call_struct_layout_matches_header(pkg, tmp_path):
    """engine.MixCall (the ctypes mirror of mx_mix_call) has the C struct's size and field offsets:
    a C program built against include/matcha_gossip.h prints them."""
    import subprocess
    import importlib
    E = importlib.import_module(pkg.__name__ + ".engine")
    fields = [f for f, _ in E.MixCall._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "matcha_gossip.h"\nint main(void) {\n'
                   '  printf("%zu", sizeof(mx_mix_call));\n'
                   + "".join(f'  printf(" %zu", offsetof(mx_mix_call, {f}));\n' for f in fields)
                   + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(E.MixCall)] + [getattr(E.MixCall, f).offset for f in fields]
    assert got == want
