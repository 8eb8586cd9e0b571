"""Build-time guard of the counted-vmcnt row kernels (CPU only: reads the gfx950
code object shipped inside libshpl.so, no GPU).

k_conv_rows and k_wgrad_rows (csrc/shpl_conv_rows.hip) stream their input rows
through a per-wave ring of LDS-DMA slots and wait for a slot with a STATIC
count, `s_waitcnt vmcnt(K) expcnt(6)` (SHPL_RING_WAIT; expcnt(6) is the
marker): K = the vector-memory operations of the RING - 1 = 2 later steps. The
wait is right only if every step issues exactly K / 2 of them. A vector-memory
operation the compiler adds (a scratch spill or reload, a hoisted load) makes
the wait stricter or a reload drain the ring; one it drops makes the MFMAs
read a slot before its DMA landed. For every instantiation in the shipped
library this test asserts:
  * no scratch: .private_segment_fixed_size 0, no VGPR spills, no scratch_*
    instruction;
  * no other vmcnt wait on those paths: the compiler's waitcnt pass does not
    see the ring's asm DMAs, so a load it still counts as pending (weights
    loaded in the prologue without a builtin wait) makes it place vmcnt waits
    down to vmcnt(0) among a step's MFMAs -- the ring drained every row;
  * every path from one marked wait to the next issues exactly K / 2 vector
    memory instructions (buffer_*, global_*, flat_*, scratch_*): uniform
    branches both ways; exec-mask branches as with active lanes (execz not
    taken, execnz taken) -- they guard the partial last DMA of a row, whose
    lane 0 is always active, and the select of a pooled piece's offset, both
    of whose sides reach the DMA.
A variant built with the waves-per-SIMD bound forced to 4
(-DSHPL_ROWS_WPE=4) spills, and the same checks must reject it.
"""
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = re.compile(r"k_conv_rowsI|k_wgrad_rowsI")
VMEM = re.compile(r"^(buffer_|global_|scratch_|flat_)")
MARK = re.compile(r"^s_waitcnt vmcnt\((\d+)\) expcnt\(6\)$")
EXIT = re.compile(r"^s_waitcnt vmcnt\(0\) expcnt\(5\)$")  # the loop's exit drain (expcnt(5): its marker)
RING = 3

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="no ROCm LLVM tools")


def gfx950_code_objects(blob):
    """The gfx950 device code objects of every offload bundle in a .hip_fatbin section (or a bundle file)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    for m in re.finditer(re.escape(magic), blob):
        s = m.start()
        n = struct.unpack_from("<Q", blob, s + len(magic))[0]
        p = s + len(magic) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                out.append(blob[s + off:s + off + size])
    return out


def library_code_objects(so):
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", so,
                        os.path.join(td, "copy.so")], check=True)
        return gfx950_code_objects(open(fb, "rb").read())


def kernel_metadata(co_path):
    """{kernel symbol: {private_segment_fixed_size, vgpr_spill_count, ...}} from the code object notes."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co_path], check=True,
                         capture_output=True, text=True).stdout
    meta, cur = {}, {}
    for line in txt.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and line.strip().startswith("-"):
            cur = {}
        cur[k] = v
        if k == "name":
            meta[v] = cur
    return meta


def disassembly(co_path):
    """{kernel symbol: [(address, instruction text)]}"""
    txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co_path], check=True,
                         capture_output=True, text=True).stdout
    out = {}
    for f in re.split(r"\n(?=[0-9a-f]+ <)", txt):
        m = re.match(r"[0-9a-f]+ <([^>]+)>", f)
        if not m:
            continue
        ins = []
        for line in f.splitlines()[1:]:
            mm = re.match(r"\s*(\S.*?)\s*//\s*([0-9A-F]+):", line)
            if mm:
                ins.append((int(mm.group(2), 16), mm.group(1)))
        out[m.group(1)] = ins
    return out


def ring_violations(name, ins):
    """Problems of one kernel's ring waits (empty list: the counted vmcnt arithmetic holds)."""
    bad = []
    if any(t.startswith("scratch_") for _, t in ins):
        bad.append("scratch instructions")
    marks = [i for i, (_, t) in enumerate(ins) if MARK.match(t)]
    if len(marks) < RING:
        return bad + [f"{len(marks)} marked ring waits (expected at least {RING})"]
    ks = {int(MARK.match(ins[i][1]).group(1)) for i in marks}
    if len(ks) != 1:
        return bad + [f"ring waits with different counts {sorted(ks)}"]
    k = ks.pop()
    per_step = k // (RING - 1)
    at = {a: i for i, (a, _) in enumerate(ins)}

    def succ(i):
        a, t = ins[i]
        op = t.split()[0]
        if op == "s_endpgm" or op == "s_setpc_b64":
            return []
        if op == "s_branch" or op.startswith("s_cbranch"):
            n = int(t.split()[1])
            n = n - 65536 if n >= 32768 else n
            tgt = at.get(a + 4 + 4 * n)
            if op == "s_cbranch_execz":  # exec-mask branches: lanes are active (see the module docstring)
                return [i + 1]
            if op == "s_cbranch_execnz":
                return [tgt]
            return [tgt] if op == "s_branch" else [tgt, i + 1]
        return [i + 1]

    mark_set = set(marks)
    counts, stray = set(), set()
    for w in marks:
        stack, seen = [(w + 1, 0)], set()
        while stack:
            i, c = stack.pop()
            if i is None or i >= len(ins) or (i, c) in seen:
                continue
            seen.add((i, c))
            t = ins[i][1]
            if i in mark_set:
                counts.add(c)
                continue
            if EXIT.match(t):  # the loop's exit drains the ring
                continue
            if t.startswith("s_waitcnt") and "vmcnt" in t:  # any other vmcnt wait drains (part of) the ring
                stray.add(t)
            if VMEM.match(t):
                c += 1
                if c > 4 * per_step:
                    counts.add(c)
                    continue
            stack.extend((s, c) for s in succ(i))
    if counts != {per_step}:
        bad.append(f"vector-memory operations between ring waits {sorted(counts)}, expected {per_step} (K={k})")
    if stray:
        bad.append(f"compiler vmcnt waits between ring waits {sorted(stray)[:4]} (they drain the ring every step)")
    return bad


def check_code_objects(cos):
    """{kernel: [problems]} over every k_conv_rows / k_wgrad_rows instantiation of the code objects."""
    report, seen = {}, 0
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(cos):
            path = os.path.join(td, f"co{n}.o")
            open(path, "wb").write(co)
            meta = kernel_metadata(path)
            dis = None
            for name, md in meta.items():
                if not KERNELS.search(name):
                    continue
                seen += 1
                bad = []
                if int(md.get("private_segment_fixed_size", "0")) != 0:
                    bad.append(f"private segment {md['private_segment_fixed_size']} B")
                if int(md.get("vgpr_spill_count", "0")) != 0:
                    bad.append(f"{md['vgpr_spill_count']} VGPR spills")
                if dis is None:
                    dis = disassembly(path)
                bad += ring_violations(name, dis.get(name, []))
                report[name] = bad
    return report, seen


def test_shipped_row_kernels_keep_the_ring_arithmetic():
    so = os.path.join(ROOT, "sparse_pooling_amd", "libshpl.so")
    if not os.path.exists(so):
        from sparse_pooling_amd import build
        build.build()
    report, seen = check_code_objects(library_code_objects(so))
    assert seen >= 40, f"found only {seen} row-kernel instantiations"
    assert any("k_wgrad_rows" in k for k in report) and any("k_conv_rows" in k for k in report)
    bad = {k: v for k, v in report.items() if v}
    assert not bad, bad


def test_guard_rejects_a_forced_spill(tmp_path):
    """The same checks on shpl_conv_rows.hip built with 4 waves per SIMD forced: spills must be caught."""
    out = tmp_path / "rows_wpe4.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "--cuda-device-only", "-DSHPL_ROWS_WPE=4", "-c",
                    os.path.join(ROOT, "sparse_pooling_amd", "csrc", "shpl_conv_rows.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    blob = out.read_bytes()
    cos = gfx950_code_objects(blob) or [blob]
    report, seen = check_code_objects(cos)
    assert seen >= 40
    flagged = [k for k, v in report.items() if any("scratch" in p or "spill" in p or "private" in p for p in v)]
    assert flagged, "a forced spill went unnoticed"


def test_guard_rejects_a_drained_ring(tmp_path):
    """The round-3 form (the prologue's weight loads left pending in the compiler's model: -DSHPL_ROWS_WLATE=1)
    has vmcnt waits among every row step's MFMAs; the checks must reject it."""
    out = tmp_path / "rows_wlate.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "--cuda-device-only", "-DSHPL_ROWS_WLATE=1", "-c",
                    os.path.join(ROOT, "sparse_pooling_amd", "csrc", "shpl_conv_rows.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    blob = out.read_bytes()
    cos = gfx950_code_objects(blob) or [blob]
    report, seen = check_code_objects(cos)
    assert seen >= 40
    flagged = [k for k, v in report.items() if any("compiler vmcnt waits" in p for p in v)]
    assert any("k_conv_rows" in k for k in flagged), "a drained ring went unnoticed"
