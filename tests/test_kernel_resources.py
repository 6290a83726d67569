"""Resource budget of the shipped gfx950 kernels, read from the built library (CPU only).

The collective kernels (ring / read / one-shot) of every rank must be resident on the
GPU at the same time: each waits for its peers' kernels.  With 8 rank processes sharing one GPU
(the reference's perf_test topology) that is 8 x 256 one-wave pipelines = 2 waves on each of
the 1024 SIMDs, so no collective kernel may use more than 256 registers per lane (VGPRs +
AGPRs); and none may use scratch memory (a spill inside the message loop costs a memory round
trip per access).  Checked from the code object's own metadata (.vgpr_count, .agpr_count,
.private_segment_fixed_size) -- no compile and no GPU needed.
"""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mini-nccl_amd", "lib", "libmini_nccl.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _gfx950_code_object(path):
    """The gfx950 entry of the clang offload bundle embedded in the library's .hip_fatbin."""
    data = open(path, "rb").read()
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    assert i >= 0, "no offload bundle in the library"
    n = struct.unpack_from("<Q", data, i + 24)[0]
    off = i + 32
    for _ in range(n):
        eo, es, idl = struct.unpack_from("<QQQ", data, off)
        tid = data[off + 24:off + 24 + idl].decode()
        off += 24 + idl
        if "gfx950" in tid and es:
            return data[i + eo:i + eo + es]
    raise AssertionError("no gfx950 code object in the bundle")


def _kernels(tmp_path):
    co = tmp_path / "co.elf"
    co.write_bytes(_gfx950_code_object(LIB))
    out = subprocess.run([READELF, "--notes", str(co)], capture_output=True, text=True, check=True).stdout
    kernels, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"\s*-?\s*\.(agpr_count|name|private_segment_fixed_size|vgpr_count):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if line.lstrip().startswith("-"):  # a new kernel record starts
            cur = {}
        if cur is None:
            continue
        cur[key] = val
        if "name" in cur and all(k in cur for k in ("agpr_count", "vgpr_count", "private_segment_fixed_size")):
            kernels[cur["name"]] = {k: int(v) for k, v in cur.items() if k != "name"}
            cur = None
    return kernels


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(READELF)), reason="library not built / no llvm-readelf")
def test_collective_kernels_fit_two_waves_per_simd_without_scratch(tmp_path):
    ks = _kernels(tmp_path)
    coll = {k: v for k, v in ks.items() if re.search(r"(ring|read|oneshot)_kernel", k)}
    # (ring, read, one-shot) x 5 dtypes x 4 ops x (vector, scalar); 6.0 dropped read's load form
    assert len(coll) == 120, sorted(coll)[:5]
    over = {k: v for k, v in coll.items() if v["vgpr_count"] + v["agpr_count"] > 256}
    assert not over, f"collective kernels above 256 registers (1 wave per SIMD): {over}"
    spill = {k: v for k, v in ks.items() if v["private_segment_fixed_size"] != 0}
    assert not spill, f"kernels using scratch memory: {spill}"


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library not built / no llvm-objdump")
def test_buffer_accesses_are_range_checked_on_their_whole_offset(tmp_path):
    # read_fold_all issues the next batch's loads unconditionally -- up to two batches
    # past the end of a slice, and so, for the last slice of a peer's chunk, past the end of the
    # peer's mapped allocation.  They touch no memory only because a raw buffer access whose
    # offset is at or past the resource's num_records returns 0 / stores nothing.  On gfx9 that
    # range check covers voffset + the instruction's immediate offset but NOT soffset: an access
    # the compiler had split into a uniform soffset part would escape it.  Every buffer load and
    # store the library ships passes soffset 0 (kernels.hip hands its whole offset to voffset).
    co = tmp_path / "co.elf"
    co.write_bytes(_gfx950_code_object(LIB))
    asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(co)], capture_output=True, text=True, check=True).stdout
    ops = [ln.split("//")[0].split() for ln in asm.splitlines() if re.match(r"\s+buffer_(load|store)_", ln)]
    assert len(ops) > 10000, len(ops)  # every kernel's buffer accesses were found
    # operands: vdata, vaddr, srsrc, soffset [, modifiers]
    bad = [" ".join(o) for o in ops if o[4].rstrip(",") != "0"]
    assert not bad, f"buffer accesses with a non-zero soffset (outside the range check): {bad[:5]}"


def _disassembly_by_kernel(tmp_path):
    co = tmp_path / "co.elf"
    co.write_bytes(_gfx950_code_object(LIB))
    asm = subprocess.run([OBJDUMP, "-d", "-C", "--mcpu=gfx950", str(co)], capture_output=True, text=True,
                         check=True).stdout
    out = {}
    for body in re.split(r"\n(?=[0-9a-f]{16} <)", asm):
        m = re.match(r"[0-9a-f]{16} <(.*)>:", body)
        if m:
            out[m.group(1)] = body
    return out


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library not built / no llvm-objdump")
def test_half_precision_sums_stay_packed(tmp_path):
    # VERDICT r5 #8, BASELINE.json configs[4] (C5: 1 GiB fp16 / bf16, "packed wavefront adds"): the
    # 16-byte paths of every Sum kernel add fp16 pairs with v_pk_add_f16 and bf16 through packed
    # f32 adds and the packed round back (v_pk_add_f32 + v_cvt_pk_bf16_f32).  A compiler change
    # that unpacks them fails here, on the CPU.
    fns = _disassembly_by_kernel(tmp_path)
    want = {  # kernel-name pattern (Sum = OPC 0, vector path) -> at least this many per kernel
        r"local_reduce_vec<{T}, 0>\(": 4,
        r"read_kernel<{T}, 0, true>\(": 16,
        r"read_grid_kernel<{T}, 0, \d, \d>\(": 4,
        r"ring_kernel<{T}, 0, true>\(": 1,
        r"oneshot_kernel<{T}, 0, true>\(": 1,
    }
    counts = {}
    for pat, least in want.items():
        for T, ops in (("_Float16", ("v_pk_add_f16",)), ("mnccl::bf16_t", ("v_pk_add_f32", "v_cvt_pk_bf16_f32"))):
            rx = re.compile(pat.replace("{T}", re.escape(T)))
            names = [k for k in fns if rx.search(k)]
            assert names, f"no kernel matches {rx.pattern}"
            for k in names:
                for op in ops:
                    c = len(re.findall(r"\s" + op + r"\b", fns[k]))
                    counts[(k, op)] = c
                    assert c >= least, f"{k}: {c} x {op} (expected >= {least})"
    assert len(counts) >= 2 * 5 * 1 + 5  # every form, both half types
