"""Static checks of the gfx950 code object inside libraftmc.so (no GPU needed).

    python scripts/check_isa.py [path/to/libraftmc.so | path/to/x.hsaco ...]

For every kernel: instruction count, long-branch sequences (s_getpc_b64 +
s_setpc_b64, emitted when a kernel outgrows the 16-bit branch range) and the
private (scratch) segment size.  Round 1 found that kernels large enough to
need long branches computed wrong results and faulted on MI355X, so the build
keeps every kernel within short-branch range and free of scratch; the CPU test
suite runs this check (tests/test_abi.py).  Round 3 adds a memory-ordering check:
no vector store or atomic may issue while a scalar load (other than of the kernel
arguments) is outstanding — the compiler reordered a counter store ahead of the
scalar load of the same counter, and the GPU intermittently lost new states.
Round 5 adds the stack check (round 4's fault: gpurun_out/r4f, an illegal address in
tlg_expand_k of the generated membership code, whose recursive perm_value ran a lane's stack
past the runtime's default per-lane stack): a generated code object may use a dynamic stack
only when its source carries the recursion marker, for which the backend raises the per-lane
stack to REC_STACK_BYTES (tlagen_backend.cpp kRecStackBytes), and no kernel's static frame may
exceed that.
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd", "_build", "libraftmc.so")
# tlagen_backend.cpp: kRecMarker (a source holding it runs with kRecStackBytes per lane)
REC_MARKER = "kMaxRecDepth) {"
REC_STACK_BYTES = 16384


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """The .hip_fatbin section holds one offload bundle per translation unit; unbundle each.
    A generated path's code object (`_build/tlagen_co/*.hsaco`, hiprtc output) is one bundle."""
    d = tempfile.mkdtemp()
    fat = os.path.join(d, "fat.bin")
    with open(lib, "rb") as f:
        raw = f.read(len(MAGIC)) == MAGIC
    if raw:
        shutil.copyfile(lib, fat)
    else:
        # objcopy without an output operand rewrites its input in place: dump from a copy, never
        # from the library a running process may have mapped
        copy = os.path.join(d, "lib.so")
        shutil.copyfile(lib, copy)
        subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, copy, os.path.join(d, "discard.so")], check=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    out = []
    for n, st in enumerate(starts):
        part = os.path.join(d, "part%d.bin" % n)
        open(part, "wb").write(blob[st:starts[n + 1] if n + 1 < len(starts) else len(blob)])
        co = os.path.join(d, "part%d.co" % n)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        out.append(co)
    return out


def kernels(co, functions=False):
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], capture_output=True,
                         text=True, check=True).stdout
    out, cur = {}, None
    smem_pending = False
    getpc_at = -99
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = {"instructions": 0, "long_branches": 0, "smem_store_hazards": 0}
            smem_pending = False
            getpc_at = -99
            continue
        if cur and line.startswith("\t"):
            out[cur]["instructions"] += 1
            # a long branch is s_getpc_b64 + offset arithmetic + s_setpc_b64; a function's return
            # is a bare s_setpc_b64 of the return address (not counted)
            if "s_getpc_b64" in line:
                getpc_at = out[cur]["instructions"]
            if "s_setpc_b64" in line and out[cur]["instructions"] - getpc_at <= 4:
                out[cur]["long_branches"] += 1
            # a scalar load from memory other than the kernel arguments (s[0:1]) still in flight
            # while a vector store / atomic is issued: the two paths are not ordered, so a store
            # to the loaded address can overtake the load (round 3: orig_advance lost counts)
            ops = line.split()
            if ops and ops[0].startswith("s_load_dword") and len(ops) > 2 and ops[2].rstrip(",") != "s[0:1]":
                smem_pending = True
            elif ops and ops[0] == "s_waitcnt" and "lgkmcnt(0)" in line:
                smem_pending = False
            elif smem_pending and ops and ops[0].startswith(("global_store", "global_atomic", "flat_store", "flat_atomic")):
                out[cur]["smem_store_hazards"] += 1
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True, text=True, check=True).stdout
    # amdhsa metadata: a list of kernel maps (keys sorted): private segment size, then symbol
    priv = re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)
    syms = re.findall(r"\.symbol:\s+(\S+)\.kd", notes)
    lds = re.findall(r"\.group_segment_fixed_size:\s+(\d+)", notes)
    dyn = re.findall(r"\.uses_dynamic_stack:\s+(\S+)", notes)
    vgpr = re.findall(r"\.vgpr_count:\s+(\d+)", notes)
    agpr = re.findall(r"\.agpr_count:\s+(\d+)", notes)
    for k, (s, p) in enumerate(zip(syms, priv)):
        if s in out:
            out[s]["scratch_bytes"] = int(p)
            if k < len(lds): out[s]["lds_bytes"] = int(lds[k])
            if k < len(vgpr): out[s]["vgprs"] = int(vgpr[k])
            if k < len(agpr): out[s]["agprs"] = int(agpr[k])
            if k < len(dyn): out[s]["dynamic_stack"] = dyn[k] == "true"
    # functions=True: device functions too (the generated path's kernels call the functions its
    # front end outlines; a long branch or store hazard inside one is as bad as in a kernel)
    return {k if "scratch_bytes" in v else "fn:" + k: v for k, v in out.items() if functions or "scratch_bytes" in v}


def stack_ok(v):
    """a kernel's stack fits what the backend gives it: a dynamic stack only in a code object whose
    source carries the recursion marker (v["raised_stack"]), and a static frame within the raised
    per-lane stack"""
    if v.get("dynamic_stack") and not v.get("raised_stack"):
        return False
    return v.get("scratch_bytes", 0) <= REC_STACK_BYTES


def violations(ks, allow_scratch=False):
    """Kernels/functions breaking the rules: long branches, store-after-scalar-load hazards, stacks the
    backend does not provide (stack_ok), and (unless allowed) scratch.  The generated path's code
    objects are allowed scratch: their kernels call outlined functions (a call stack) and keep a
    state's variable handles in a private array; the hand-compiled library is not."""
    return {k: v for k, v in ks.items()
            if v["long_branches"] or v["smem_store_hazards"] or (not allow_scratch and v.get("scratch_bytes")) or not stack_ok(v)}


def raised_stack(hsaco):
    """True when the generated source of this code object (a *.gen.hip next to it whose cache key is
    the file name, prebuild.py key_of) carries the recursion marker"""
    d = os.path.dirname(os.path.abspath(hsaco))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd", "csrc", "tlagen"))
    from prebuild import key_of
    want = os.path.basename(hsaco)[:-len(".hsaco")]
    for f in os.listdir(d):
        if f.endswith(".gen.hip"):
            src = open(os.path.join(d, f)).read()
            if key_of(src) == want:
                return REC_MARKER in src
    return False


def main():
    libs = sys.argv[1:] or [DEFAULT]
    gen = all(l.endswith(".hsaco") for l in libs)
    ks = {}
    for lib in libs:
        raised = lib.endswith(".hsaco") and raised_stack(lib)
        for co in code_objects(lib):
            for k, v in kernels(co, gen).items():
                v["raised_stack"] = raised
                ks[k if len(libs) == 1 else os.path.basename(lib) + ":" + k] = v
    print(json.dumps(ks, indent=1, sort_keys=True))
    return 1 if violations(ks, allow_scratch=gen) else 0


if __name__ == "__main__":
    sys.exit(main())
