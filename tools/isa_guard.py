#!/usr/bin/env python3
"""Call check over the SHIPPED gfx950 code objects (lib/libzkalgebra_gpu.so's .hip_fatbin).

Round 4's first Jacobian group-FFT build hung the GPU: `xyzz_scl` was left outlined (a real
call, `s_swappc_b64 s[30:31], ...` into it and `s_setpc_b64 s[30:31]` back), and LLVM's branch
relaxation expanded a long branch inside the callee with s[30:31] -- the return address -- as its
scratch pair, unsaved, so the function's return jumped back into its own body and the kernel
never finished (profiles/r05a_fft_outlined_scl.txt: the excerpt of that variant's assembly).
The fix forces every point routine inline.  This checker keeps it that way:

  * no code object of the library may contain a call (`s_swappc_b64`) -- every device function
    is inlined into its kernel, so there is no return address to clobber;
  * every `s_setpc_b64` must end the long-branch idiom `s_getpc_b64 sP` / `s_add_u32` /
    `s_addc_u32` / `s_setpc_b64 sP` with the same pair, and that pair must not be s[30:31].

    python tools/isa_guard.py [lib.so]       # prints a summary, exit 1 on a violation
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "zikkurat-algebra_amd", "lib", "libzkalgebra_gpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib=LIB):
    """the gfx950 device ELF images of every offload bundle in the library's .hip_fatbin"""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin",
                               lib, fb])
        data = open(fb, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        s = m.start()
        n = struct.unpack_from("<Q", data, s + len(MAGIC))[0]
        p = s + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple and size:
                out.append(data[s + off:s + off + size])
    return out


def disassemble(image):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(image)
        f.flush()
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", f.name],
                              check=True, capture_output=True, text=True).stdout


def functions(text):
    """{symbol: [instruction lines]} of an llvm-objdump -d listing, or of compiler assembly (-S)"""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line) or re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        s = line.strip()
        if cur is None or not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        s = re.sub(r"^[0-9a-f]+:\s*", "", s)  # objdump address column
        s = s.split("//")[0].split(";")[0].strip()
        if s:
            funcs[cur].append(s)
    return funcs


def violations(funcs):
    """(function, reason) for every call and every s_setpc_b64 outside the long-branch idiom or
    through the return-address pair s[30:31]"""
    bad = []
    for name, ins in funcs.items():
        for i, s in enumerate(ins):
            op = s.split()[0]
            if op == "s_swappc_b64":
                bad.append((name, f"call: {s}"))
            elif op == "s_getpc_b64" and s.split()[1] == "s[30:31]":
                bad.append((name, f"long branch built in the return-address pair: {s}"))
            elif op == "s_setpc_b64":
                pair = s.split()[1]
                if pair == "s[30:31]":
                    bad.append((name, f"s_setpc_b64 through the return-address pair: {s}"))
                    continue
                prev = ins[max(0, i - 4):i]
                if not any(p.split()[0] == "s_getpc_b64" and p.split()[1].rstrip(",") == pair for p in prev):
                    bad.append((name, f"s_setpc_b64 outside a long-branch idiom: {s}"))
    return bad


def check(lib=LIB):
    """-> (number of kernels, names of group-FFT kernels seen, violations)"""
    kernels, fft, bad = 0, [], []
    for image in code_objects(lib):
        funcs = functions(disassemble(image))
        kernels += len(funcs)
        fft += [f for f in funcs if re.search(r"k_fft_|k_subgroup_check", f)]
        bad += violations(funcs)
    return kernels, fft, bad


if __name__ == "__main__":
    n, fft, bad = check(sys.argv[1] if len(sys.argv) > 1 else LIB)
    print(f"{n} device functions, {len(fft)} group-FFT kernels, {len(bad)} violations")
    for name, why in bad[:20]:
        print(f"  {name}: {why}")
    sys.exit(1 if bad else 0)
