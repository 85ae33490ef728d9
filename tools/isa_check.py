"""Scan the gfx950 assembly of the HIP sources for two instruction patterns kept out of every kernel:

  * packed-FP32 ops (v_pk_fma/mul/add_f32) whose LOW lane reads the HIGH element of a source (an
    op_sel bit set; VGPR or SGPR pair) in a kernel that also runs MFMAs.  Such ops returned wrong
    low-lane values in lanes 48-63 now and then while another wave of the workgroup ran MFMAs
    (k_fused_proj, round 2: dump instances of the kernel found the corrupted X values, all from
    `v_pk_fma_f32 ... op_sel:[1,0,0]`; tests/test_gpu_proj_fused.py::test_repeatable_under_poisoned_memory re-runs the poisoned-memory repro; with
    the broadcasts materialised by splat2() 0 of 220 poisoned runs differ, against ~4 % before).
    Round 3: SGPR-pair broadcasts (the epilogue scale of the build and fused kernels) are held to the
    same rule -- they were bit-exact in every test, but the guard no longer rests on that;
  * MFMAs whose destination overlaps their own A or B source registers (reported, not fatal);
  * (round 4, the library scan) scratch use in the kernels whose operand loads are hidden from the compiler's
    s_waitcnt bookkeeping (inline-asm loads into VGPRs, waited for by counted s_waitcnt: k_build_f32r,
    k_build_bf16_2b, k_build_bf16).  Those are correct only while the destination registers are never spilled:
    a spill would store a register before its load has landed (the round-1 fault of k_build_bf16_2b<32>).  A
    non-zero private segment, VGPR or SGPR spill count there fails the check; `--resources` lists every
    kernel's VGPRs / AGPRs / LDS / scratch.

    python tools/isa_check.py                 the shipped dvccorr/libdvccorr.so (seconds: its gfx950 code
                                              objects are unbundled and disassembled)
    python tools/isa_check.py file.hip ...    recompile those sources to assembly instead
    exit status 1 if such an op_sel read is found"""
import concurrent.futures as cf
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raft-dvc_amd", "csrc")
MF = re.compile(r'v_mfma\S+\s+v\[(\d+):(\d+)\],\s+v\[(\d+):(\d+)\],\s+v\[(\d+):(\d+)\]')
PK = re.compile(r'v_pk_(?:fma|mul|add)_f32\b.*\bop_sel:\[([01,]+)\]')


def extra_flags(src):
    """Per-object flags of the Makefile ('obj/X.o: EXTRA := ...')."""
    obj = "obj/" + os.path.splitext(os.path.basename(src))[0] + ".o"
    for line in open(os.path.join(CSRC, "Makefile")):
        m = re.match(r'^(\S+):\s*EXTRA\s*:=\s*(.*)$', line)
        if m and m.group(1) == obj:
            return m.group(2).split()
    return []


def assemble(src, tmp):
    out = os.path.join(tmp, os.path.basename(src) + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + CSRC, "--cuda-device-only", "-S", src, "-o", out] + extra_flags(src), check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return out


def opsel_read(line, bits):
    """True if a source whose op_sel bit is set is a register pair (VGPR or SGPR): its high element
    feeds the low lane.  (A literal / inline constant with op_sel set reads no register half.)"""
    ops = [o.strip() for o in line.split("//")[0].split(None, 1)[1].split(" op_sel")[0].split(",")]
    srcs = ops[1:]   # ops[0] is the destination
    return any(b == "1" and i < len(srcs) and srcs[i][:1] in ("v", "s") for i, b in enumerate(bits.split(",")))


LLVM = "/opt/rocm/llvm/bin"
LIB = os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr.so")


def disassemble_library(lib, tmp):
    """One disassembly file per offload bundle of the library's .hip_fatbin (one bundle per source)."""
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section", ".hip_fatbin=" + fb, lib, os.path.join(tmp, "lib.copy")],
                   check=True)
    data = open(fb, "rb").read()
    offs = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)] + [len(data)]
    outs = []
    for i in range(len(offs) - 1):
        b, co, dis = (os.path.join(tmp, f"b{i}.{x}") for x in ("bin", "co", "s"))
        open(b, "wb").write(data[offs[i]:offs[i + 1]])
        subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + b,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        with open(dis, "w") as f:
            subprocess.run([LLVM + "/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, stdout=f)
        outs.append(dis)
    return outs


def check_library(lib=LIB):
    with tempfile.TemporaryDirectory() as tmp:
        return {f"bundle{i}": scan(d) for i, d in enumerate(disassemble_library(lib, tmp))}


# kernels whose VGPR operand loads are issued from inline asm (invisible to the compiler's waitcnt insertion):
# every k_build_f32r, and k_build_bf16 / k_build_bf16_2b with NCH <= 16 (build_gemm.hip Hidden<NCH>; the NCH = 32
# instances load through the compiler and may spill)
HIDDEN_LOAD_KERNELS = re.compile(r'k_build_f32r|k_build_bf16_2bILi(?:4|8|16)E|k_build_bf16ILi(?:4|8|16)E')
RES_KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
            ".private_segment_fixed_size", ".group_segment_fixed_size")


def kernel_resources(lib=LIB):
    """{kernel symbol: {key: int}} from the AMDGPU metadata notes of every gfx950 code object in the library."""
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        fb = os.path.join(tmp, "fatbin")
        subprocess.run([LLVM + "/llvm-objcopy", "--dump-section", ".hip_fatbin=" + fb, lib, os.path.join(tmp, "c")],
                       check=True)
        data = open(fb, "rb").read()
        offs = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)] + [len(data)]
        for i in range(len(offs) - 1):
            b, co = os.path.join(tmp, f"b{i}.bin"), os.path.join(tmp, f"b{i}.co")
            open(b, "wb").write(data[offs[i]:offs[i + 1]])
            subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + b,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
            notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            cur = {}
            for line in notes.splitlines():
                t = line.strip().lstrip("- ").strip()
                for k in RES_KEYS:
                    if t.startswith(k + ":"):
                        cur[k] = int(t.split(":", 1)[1])
                if t.startswith(".name:"):
                    cur["name"] = t.split(":", 1)[1].strip()
                if t.startswith(".wavefront_size:") and "name" in cur:   # last key of a kernel's record
                    res[cur.pop("name")] = cur
                    cur = {}
    return res


def spill_violations(res):
    """Hidden-load kernels with scratch, VGPR or SGPR spills."""
    return {k: v for k, v in res.items() if HIDDEN_LOAD_KERNELS.search(k) and
            (v.get(".private_segment_fixed_size", 0) or v.get(".vgpr_spill_count", 0) or v.get(".sgpr_spill_count", 0))}


def scan(asm):
    """(op_sel reads in kernels that also run MFMAs, MFMA overlaps, op_sel reads in MFMA-free kernels,
    names of the kernels that run MFMAs)"""
    pk, mf, has_mfma = {}, {}, set()
    cur = None
    for line in open(asm):
        m = re.match(r'^(_Z\S+):', line) or re.match(r'^[0-9a-f]+ <(_Z\S+)>:', line)
        if m:
            cur = m.group(1)
            continue
        if "v_mfma" in line:
            has_mfma.add(cur)
        m = PK.search(line)
        if m and "1" in m.group(1) and opsel_read(line, m.group(1)):
            pk.setdefault(cur, []).append(line.strip())
        m = MF.search(line)
        if m:
            r = [int(g) for g in m.groups()]
            d = set(range(r[0], r[1] + 1))
            if d & (set(range(r[2], r[3] + 1)) | set(range(r[4], r[5] + 1))):
                mf.setdefault(cur, []).append(line.strip())
    return ({k: v for k, v in pk.items() if k in has_mfma}, mf,
            {k: v for k, v in pk.items() if k not in has_mfma}, has_mfma)


def check(files):
    with tempfile.TemporaryDirectory() as tmp, cf.ThreadPoolExecutor(max_workers=8) as ex:
        asms = list(ex.map(lambda f: assemble(f, tmp), files))
        return {os.path.basename(f): scan(a) for f, a in zip(files, asms)}


if __name__ == "__main__":
    if sys.argv[1:2] == ["--resources"]:
        for k, v in sorted(kernel_resources().items(), key=lambda kv: kv[0]):
            print(f"{k[:90]:90s} vgpr {v.get('.vgpr_count')} agpr {v.get('.agpr_count')} "
                  f"lds {v.get('.group_segment_fixed_size')} scratch {v.get('.private_segment_fixed_size')} "
                  f"spill {v.get('.vgpr_spill_count')}/{v.get('.sgpr_spill_count')}")
        sys.exit(0)
    res = check(sys.argv[1:]) if sys.argv[1:] else check_library()
    if not sys.argv[1:]:
        rv = kernel_resources()
        bad = spill_violations(rv)
        hidden = [k for k in rv if HIDDEN_LOAD_KERNELS.search(k)]
        print(f"hidden-load kernels checked for spills: {len(hidden)}; with scratch / spills: {len(bad)}")
        for k, v in bad.items():
            print(f"  SPILL in hidden-load kernel {k[:80]}: {v}")
        if bad:
            sys.exit(1)
    npk = 0
    for f, (pk, mf, quiet, _) in res.items():
        for k, v in pk.items():
            npk += len(v)
            print(f"{f}: {k[:70]}: {len(v)} packed-FP32 op_sel reads beside MFMAs, e.g. {v[0]}")
        for k, v in quiet.items():
            print(f"{f}: {k[:70]}: {len(v)} packed-FP32 op_sel reads, no MFMA in the kernel (informational)")
        for k, v in mf.items():
            print(f"{f}: {k[:70]}: {len(v)} MFMA dst/src overlaps (informational)")
    print("packed-FP32 op_sel reads in kernels with MFMAs:", npk)
    sys.exit(1 if npk else 0)
