"""Host-side AddressSanitizer pass over the C ABI (CPU only, no GPU needed).

Builds every libppox translation unit with the host half under -fsanitize=address (device code is
compiled as usual), generates a driver from include/ppox.h that calls EVERY entry point twice —
all arguments zero / null, and null pointers with sizes 16 — and runs it: each call must return
(validation errors are expected and their message is read back through ppox_last_error), and ASan
must report nothing in the host shims (argument checks, workspace-size arithmetic, the error
channel).  Without a GPU no kernel runs: calls that pass validation fail at the launch.
Usage: python tools/asan_abi.py [outdir]   (exit status 0 = clean)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def declarations():
    text = open(os.path.join(ROOT, "include", "ppox.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = []
    for m in re.finditer(r"^(int|int64_t|int32_t|const char\*)\s+(ppox_\w+)\(([^;]*?)\);", text, flags=re.M | re.S):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        decls.append((ret, name, params))
    return decls


def arg(param, sized):
    t = param.rsplit(" ", 1)[0] if " " in param else param
    if "*" in param:
        return "nullptr"
    if "double" in t or "float" in t:
        return "0.5" if sized else "0"
    return "16" if sized else "0"


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/ppox_asan"
    os.makedirs(out, exist_ok=True)
    decls = declarations()
    lines = ['#include <cstdio>', '#include "ppox.h"', "int main() {", "    int n = 0;"]
    for ret, name, params in decls:
        for sized in (False, True):
            call = f"{name}({', '.join(arg(p, sized) for p in params)})"
            if ret == "const char*":
                lines.append(f"    {{ const char* s = {call}; n += s != nullptr; }}")
            else:
                lines.append(f"    {{ long long r = (long long){call}; const char* e = ppox_last_error(); "
                             f"n += (r != 0) + (e && e[0]); }}")
    lines += [f'    std::printf("asan_abi: %d entry points called twice, %d nonzero results / messages\\n", '
              f'{len(decls)}, n);', "    return 0;", "}"]
    drv = os.path.join(out, "driver.cpp")
    open(drv, "w").write("\n".join(lines) + "\n")
    src = os.path.join(ROOT, "ppo-exploration_amd", "csrc")
    flags = ["-O1", "-g", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-munsafe-fp-atomics",
             "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include")]
    objs, procs = [], []
    for f in sorted(os.listdir(src)):
        if f.endswith((".hip", ".cpp")):
            o = os.path.join(out, f + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([HIPCC] + flags + ["-c", os.path.join(src, f), "-o", o]))
    if any(p.wait() for p in procs):
        sys.exit("asan_abi: build failed")
    exe, dobj = os.path.join(out, "asan_abi"), os.path.join(out, "driver.o")
    subprocess.check_call(["g++", "-fsanitize=address", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                           "-c", drv, "-o", dobj])
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-fsanitize=address", dobj] + objs + ["-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([exe], env=env, capture_output=True, text=True)
    sys.stdout.write(r.stdout[-2000:])
    sys.stderr.write(r.stderr[-4000:])
    if r.returncode != 0 or "ERROR: AddressSanitizer" in r.stderr:
        sys.exit(f"asan_abi: FAILED (exit {r.returncode})")
    print(f"asan_abi: clean ({len(decls)} entry points)")


if __name__ == "__main__":
    main()
