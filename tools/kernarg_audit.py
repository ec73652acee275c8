#!/usr/bin/env python3
"""Kernel-argument and private-segment audit of the engine's gfx950 code objects (test
infrastructure; tests/test_kernarg_audit.py runs it on every object of the library).

Per kernel it reports:
  - `.private_segment_fixed_size` (scratch bytes per lane, from the code object metadata) and
    whether any scratch access is NOT a register spill/reload (i.e. a stack array);
  - every VECTOR-memory access whose address derives from the kernarg segment pointer: a VALU
    instruction that reads the kernarg SGPR pair (or a copy of it), or a global/buffer/flat access
    that takes it as its scalar base.

The second is the construct behind round 5's non-deterministic decrypt misreads:
indexing a by-value argument array (`Bounds::b[i]`) with a lane-varying i makes the compiler read
the kernarg segment through the vector memory path (`v_lshl_add_u64 v, v, 2, s[0:1]` +
`global_load_dword ... offset:80`) instead of with scalar loads.  The engine's kernels read their
arguments with s_load only, so the audit must find none.

Inputs: compiler assembly (`hipcc --cuda-device-only -S`, or `--save-temps`' `*-gfx950.s`), or a
host object / library built by hipcc (`build/*.o`): its `.hip_fatbin` bundle is unpacked with
clang-offload-bundler and disassembled with llvm-objdump, and the kernel descriptors are decoded
from the code object's symbol table.

Heuristic by design: the kernarg pair (and SGPR copies of it) is tracked in program order from the
kernel's entry until every tracked SGPR has been overwritten; control flow is not followed.

usage: kernarg_audit.py FILE.{s,o} [...]   (exit 1 if any kernel reads its arguments per lane)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_REG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
# SALU mnemonics whose first operand is NOT a destination
# (the engine's kernels have no scalar-memory writes at all; any other SALU with a first operand
# in the tracked pair just ends the tracking of those SGPRs, which is conservative)
_SALU_NODEST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_setprio", "s_nop",
                "s_endpgm", "s_barrier", "s_sleep", "s_sendmsg", "s_trap", "s_icache", "s_setreg",
                "s_set_gpr_idx", "s_wait", "s_getpc", "s_setpc")


def _sgprs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _split_ops(rest):
    rest = rest.split("//")[0].split(";")[0].strip()
    return [o.strip() for o in rest.split(",")] if rest else []


def _metadata(lines):
    """kernel name -> private_segment_fixed_size, from the YAML metadata (.s or readelf --notes)"""
    meta, cur = {}, None
    for ln in lines:
        m = re.match(r"\s+\.name:\s+(\S+)", ln)
        if m:
            cur = m.group(1)
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", ln)
        if m and cur:
            meta[cur] = int(m.group(1))
    return meta


def _audit_body(body, k):
    """body: instruction lines of one kernel in program order; k: first kernarg SGPR"""
    live, findings, scratch_nonspill = {k, k + 1}, [], 0
    for ln in body:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        mn, _, rest = t.partition(" ")
        if mn.startswith("scratch_") and not re.search(r"Spill|Reload", t):
            scratch_nonspill += 1
        ops = _split_ops(rest)
        if not ops or not live:
            continue
        if mn.startswith("v_"):
            # VALU: a scalar destination (readfirstlane, cmp_e64, carry-outs) overwrites it
            dst = _sgprs(ops[0])
            first_src = 1
            if mn.startswith(("v_mad_u64_u32", "v_mad_i64_i32", "v_div_scale")) or "_co_" in mn \
                    or mn.startswith(("v_addc_", "v_subb_", "v_subbrev_")):
                if len(ops) > 1 and _sgprs(ops[1]) & live:
                    live -= _sgprs(ops[1])  # VOP3b carry-out written into a tracked SGPR
                    continue
                first_src = 2
            srcs = set().union(*(_sgprs(o) for o in ops[first_src:])) if len(ops) > first_src else set()
            if mn.startswith(("v_cmp_", "v_readfirstlane", "v_readlane")) and dst & live:
                live -= dst
                continue
            if srcs & live or (not mn.startswith(("v_cmp_", "v_readfirstlane", "v_readlane"))
                               and dst & live and not mn.startswith("v_writelane")):
                findings.append(t.split("//")[0].strip())
        elif mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
            if set().union(*(_sgprs(o) for o in ops)) & live:
                findings.append(t.split("//")[0].strip())
        elif mn.startswith("s_") and not mn.startswith(_SALU_NODEST):
            dst = _sgprs(ops[0])
            if mn in ("s_mov_b64", "s_mov_b32") and len(ops) > 1 and _sgprs(ops[1]) & live:
                live |= dst  # a copy of the kernarg pointer is tracked too
            elif dst & live:
                live -= dst  # these SGPRs are reused from here on
    return findings, scratch_nonspill


def parse_asm(path):
    """-> {kernel: {"private", "kernarg_sgpr", "findings", "scratch_nonspill"}} from compiler .s"""
    lines = open(path).read().splitlines()
    meta = _metadata(lines)
    res = {}
    for i, ln in enumerate(lines):
        m = re.match(r"\s*\.amdhsa_kernel\s+(\S+)", ln)
        if not m:
            continue
        name, fields = m.group(1), {}
        for ln2 in lines[i + 1:]:
            if ".end_amdhsa_kernel" in ln2:
                break
            m2 = re.match(r"\s*\.amdhsa_(\S+)\s+(\S+)", ln2)
            if m2:
                fields[m2.group(1)] = m2.group(2)
        if fields.get("user_sgpr_kernarg_segment_ptr") != "1":
            continue
        k = 4 * int(fields.get("user_sgpr_private_segment_buffer", "0")) \
            + 2 * int(fields.get("user_sgpr_dispatch_ptr", "0")) \
            + 2 * int(fields.get("user_sgpr_queue_ptr", "0"))
        start = next((j for j, l in enumerate(lines) if l.startswith(name + ":")), None)
        if start is None:
            continue
        body = []
        for l in lines[start + 1:]:
            if l.startswith(".Lfunc_end"):
                break
            body.append(l)
        f, ns = _audit_body(body, k)
        res[name] = {"private": meta.get(name, -1), "kernarg_sgpr": k, "findings": f,
                     "scratch_nonspill": ns}
    return res


def _elf_symbols(blob):
    """ELF64 LE: [(name, value, size)] of .symtab, and [(addr, offset, size)] of the sections"""
    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", blob, 0x3A)
    secs = []
    for i in range(shnum):
        sh = struct.unpack_from("<IIQQQQIIQQ", blob, shoff + i * shentsize)
        secs.append(sh)
    syms = []
    for sh in secs:
        if sh[1] != 2:  # SHT_SYMTAB
            continue
        strsec = secs[sh[6]]
        for j in range(sh[5] // 24):
            st_name, _, _, _, st_value, st_size = struct.unpack_from("<IBBHQQ", blob, sh[4] + 24 * j)
            s0 = strsec[4] + st_name
            name = blob[s0:blob.index(b"\0", s0)].decode()
            syms.append((name, st_value, st_size))
    return syms, [(sh[3], sh[4], sh[5]) for sh in secs if sh[3]]


def parse_object(path):
    """the same from a hipcc-built host object: unbundle, decode the kernel descriptors, disassemble"""
    secs = subprocess.run([f"{LLVM}/llvm-readelf", "-S", path], check=True, capture_output=True,
                          text=True).stdout
    if ".hip_fatbin" not in secs:
        return {}  # host-only translation unit (no device code)
    with tempfile.TemporaryDirectory() as tmp:
        fb, co = os.path.join(tmp, "fb"), os.path.join(tmp, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path,
                        os.path.join(tmp, "host")], check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                        f"--output={co}"], check=True, capture_output=True)
        blob = open(co, "rb").read()
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout.splitlines()
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                             capture_output=True, text=True).stdout.splitlines()
    meta = _metadata(notes)
    syms, secs = _elf_symbols(blob)
    kds = {}
    for name, value, size in syms:
        if not name.endswith(".kd") or size != 64:
            continue
        off = next(o + value - a for a, o, s in secs if a <= value < a + s)
        props, = struct.unpack_from("<H", blob, off + 56)  # kernel_code_properties
        if props & (1 << 3):  # ENABLE_SGPR_KERNARG_SEGMENT_PTR
            kds[name[:-3]] = 4 * (props & 1) + 2 * ((props >> 1) & 1) + 2 * ((props >> 2) & 1)
    bodies, cur = {}, None
    for ln in dis:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            cur = m.group(1)
            bodies[cur] = []
        elif cur is not None:
            bodies[cur].append(ln)
    res = {}
    for name, k in kds.items():
        f, _ = _audit_body(bodies.get(name, []), k)
        # (objdump prints no spill comments: scratch accesses are not classified here)
        res[name] = {"private": meta.get(name, -1), "kernarg_sgpr": k, "findings": f,
                     "scratch_nonspill": None}
    return res


def parse(path):
    return parse_asm(path) if path.endswith(".s") else parse_object(path)


def main(argv):
    bad = 0
    for path in argv:
        for name, r in sorted(parse(path).items()):
            tag = "OK " if not r["findings"] else "BAD"
            bad += bool(r["findings"])
            print(f"{tag} private={r['private']:4d} {name}")
            for t in r["findings"][:4]:
                print(f"      {os.path.basename(path)}: {t}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
