"""The Go binding (go/rtgpu, go/rt) against include/rtgpu.h and the reference.

There is no Go toolchain in this image, so the cgo files are compile-
unverified; these tests pin what a compile would catch and what a compile
would NOT catch (layout drift, which cgo only reports through the size
asserts at the bottom of rtgpu.go):

* every mirror struct (`//rtgpu:mirror <c type>`) has the offset and size of
  each tagged field, and the total size, that gcc gives the C struct;
* every `Kind*/Mat*/Tex*/Status*/Opt*/Build*` constant equals the C enum
  value its comment names, and ABIVersion equals RT_ABI_VERSION;
* every `C.<name>` the binding uses is declared in rtgpu.h (or is libc/cgo);
* the in-package files only select fields and methods that the reference's
  own types declare (rt/*.go), and only call functions defined in the
  reference's package rt, in the binding itself, or Go builtins (skipped
  when /root/reference is absent).
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTGPU_GO = os.path.join(ROOT, "go", "rtgpu", "rtgpu.go")
RT_DIR = os.path.join(ROOT, "go", "rt")
HEADER = os.path.join(ROOT, "include", "rtgpu.h")
REFERENCE_RT = "/root/reference/rt"

GO_SCALARS = {"int8": 1, "uint8": 1, "byte": 1, "int16": 2, "uint16": 2, "int32": 4, "uint32": 4, "float32": 4,
              "int64": 8, "uint64": 8, "float64": 8}


def _read(p):
    with open(p) as f:
        return f.read()


def _go_type(t):
    """(size, align) of a Go scalar or (nested) array type on amd64."""
    m = re.fullmatch(r"\[(\d+)\](.+)", t)
    if m:
        s, a = _go_type(m.group(2))
        return int(m.group(1)) * s, a
    s = GO_SCALARS[t]
    return s, s


def parse_mirrors(src):
    """{go name: (c name, [(go field, c field, offset, size)], size)}."""
    out = {}
    for m in re.finditer(r"//rtgpu:mirror (\w+)\ntype (\w+) struct \{\n(.*?)\n\}", src, re.S):
        cname, gname, body = m.groups()
        off, align_max, fields = 0, 1, []
        for line in body.splitlines():
            fm = re.match(r"\s*(\w+)\s+(\S+)\s+`c:\"([\w-]+)\"`", line)
            assert fm, f"{gname}: unparsed field line {line!r}"
            name, typ, cf = fm.groups()
            size, align = _go_type(typ)
            off = (off + align - 1) // align * align
            fields.append((name, cf, off, size))
            off += size
            align_max = max(align_max, align)
        out[gname] = (cname, fields, (off + align_max - 1) // align_max * align_max)
    return out


def _compile_and_run(csrc, tmp):
    c = os.path.join(tmp, "probe.c")
    exe = os.path.join(tmp, "probe")
    with open(c, "w") as f:
        f.write(csrc)
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True,
                   capture_output=True)
    return subprocess.run([exe], check=True, capture_output=True, text=True).stdout


def test_mirror_structs_match_the_header():
    mirrors = parse_mirrors(_read(RTGPU_GO))
    # everything package rt fills and rtgpu passes by pointer must be mirrored
    assert {"Node", "Material", "Texture", "Perlin", "CameraDesc", "Bucket", "Stats", "SceneInfo"} <= set(mirrors)
    assert mirrors["Node"][2] == 192          # rt_hittable
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "rtgpu.h"', "int main(void) {"]
    for g, (cname, fields, _) in mirrors.items():
        lines.append(f'  printf("{g} size %zu\\n", sizeof({cname}));')
        for name, cf, _, _ in fields:
            if cf == "-":
                continue
            lines.append(f'  printf("{g}.{name} %zu %zu\\n", offsetof({cname}, {cf}), sizeof((({cname}*)0)->{cf}));')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as tmp:
        out = _compile_and_run("\n".join(lines) + "\n", tmp)
    c = {}
    for line in out.splitlines():
        k, *v = line.split()
        c[k] = tuple(int(x) for x in v[-2:]) if v[0] != "size" else int(v[1])
    covered = 0
    for g, (cname, fields, size) in mirrors.items():
        assert c[g] == size, f"{g}: Go size {size} != sizeof({cname}) {c[g]}"
        for name, cf, off, fsize in fields:
            if cf == "-":
                continue
            assert c[f"{g}.{name}"] == (off, fsize), f"{g}.{name}: Go (offset, size) {(off, fsize)} != C {c[f'{g}.{name}']}"
            covered += 1
    assert covered >= 70


def test_mirror_covers_every_c_field():
    """A field added to a C struct must be added to its Go mirror."""
    hdr = _read(HEADER)
    for g, (cname, fields, _) in parse_mirrors(_read(RTGPU_GO)).items():
        m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), hdr, re.S)
        assert m, cname
        body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
        cfields = set()
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
            for n in names.split(","):
                cfields.add(re.match(r"\s*\**\s*(\w+)", n).group(1))
        mirrored = {cf for _, cf, _, _ in fields if cf != "-"}
        assert mirrored == cfields, f"{g} vs {cname}: missing {cfields - mirrored}, extra {mirrored - cfields}"


def test_constants_match_the_c_enums():
    src = _read(RTGPU_GO)
    consts = re.findall(r"^\s*(\w+)\s+(?:int32\s+)?=\s*(-?\d+)\s*//\s*(RT_\w+)", src, re.M)
    assert len(consts) >= 35
    lines = ["#include <stdio.h>", '#include "rtgpu.h"', "int main(void) {"]
    for name, _, cn in consts:
        lines.append(f'  printf("{name} %d\\n", (int)({cn}));')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as tmp:
        out = _compile_and_run("\n".join(lines) + "\n", tmp)
    c = dict(line.split() for line in out.splitlines())
    for name, v, cn in consts:
        assert int(c[name]) == int(v), f"{name} = {v} but {cn} = {c[name]}"


def test_c_identifiers_exist():
    src = _read(RTGPU_GO)
    hdr = _read(HEADER)
    libc = {"calloc", "free", "int", "int32_t", "uint32_t", "uint8_t", "double", "float", "size_t", "GoString"}
    used = set(re.findall(r"\bC\.(\w+)", src))
    assert used
    for name in sorted(used):
        if name in libc:
            continue
        bare = name[len("sizeof_"):] if name.startswith("sizeof_") else name
        assert re.search(r"\b%s\b" % bare, hdr), f"C.{name} is not declared in rtgpu.h"


# ---- the in-package files against the reference's package rt ---------------

GO_BUILTINS = {"append", "cap", "copy", "len", "make", "max", "min", "new", "panic", "print", "println", "delete",
               "int", "int32", "int64", "uint32", "uint64", "float32", "float64", "byte", "string", "uintptr", "bool",
               "func", "if", "for", "switch", "return", "range"}


def _ref_decls():
    types, funcs, methods = {}, set(), {}
    for fn in os.listdir(REFERENCE_RT):
        if not fn.endswith(".go"):
            continue
        src = _read(os.path.join(REFERENCE_RT, fn))
        for m in re.finditer(r"^type (\w+) struct \{\n(.*?)\n\}", src, re.S | re.M):
            fields = set()
            for line in m.group(2).splitlines():
                line = line.split("//")[0].strip()
                if not line:
                    continue
                fm = re.match(r"(\w+(?:\s*,\s*\w+)*)\s+\S", line)
                if fm:
                    fields |= {n.strip() for n in fm.group(1).split(",")}
                else:
                    fields.add(line.lstrip("*").split(".")[-1])   # embedded
            types[m.group(1)] = fields
        for m in re.finditer(r"^type (\w+) ", src, re.M):
            types.setdefault(m.group(1), set())
        funcs |= set(re.findall(r"^func (\w+)\(", src, re.M))
        for recv, name in re.findall(r"^func \(\w+ \*?(\w+)\) (\w+)\(", src, re.M):
            methods.setdefault(recv, set()).add(name)
    return types, funcs, methods


@pytest.mark.skipif(not os.path.isdir(REFERENCE_RT), reason="reference tree not present")
def test_flattener_selects_only_reference_fields():
    types, funcs, methods = _ref_decls()
    src = _read(os.path.join(RT_DIR, "gpu_flatten.go"))
    # case *T: blocks of the type switches: o.<sel> must be a field or method of T
    checked = 0
    for m in re.finditer(r"case \*(\w+):(.*?)(?=\n\s*case |\n\s*default:)", src, re.S):
        t, body = m.groups()
        assert t in types, f"reference has no type {t}"
        for sel in set(re.findall(r"\bo\.(\w+)", body)):
            assert sel in types[t] or sel in methods.get(t, set()), f"{t} has no field or method {sel}"
            checked += 1
    assert checked >= 40
    # selectors outside the switches
    for sel in set(re.findall(r"\bc\.(\w+)", src.split("func GPUCameraDesc")[1])):
        assert sel in types["Camera"] | methods.get("Camera", set()), f"Camera has no {sel}"
    for sel in set(re.findall(r"\benv\.(\w+)", src)):
        assert sel in types["HDRIEnvironment"] | methods.get("HDRIEnvironment", set()), sel
    for sel in set(re.findall(r"\bimg\.(\w+)", src)):
        assert sel in types["ImageLoader"] | methods.get("ImageLoader", set()), sel
    for sel in set(re.findall(r"\bp\.(\w+)", src.split("func (f *gpuFlat) perlin")[1].split("\nfunc ")[0])):
        assert sel in types["Perlin"], sel


@pytest.mark.skipif(not os.path.isdir(REFERENCE_RT), reason="reference tree not present")
def test_renderer_uses_only_bucket_renderer_members():
    types, funcs, methods = _ref_decls()
    src = _read(os.path.join(RT_DIR, "gpu_bucket_renderer.go"))
    br = types["BucketRenderer"] | methods.get("BucketRenderer", set())
    used = set(re.findall(r"\br\.(\w+)", src))
    assert {"framebuffer", "mu", "completed", "currentPass", "totalPasses", "passComplete"} <= used
    for sel in used:
        assert sel in br, f"BucketRenderer has no {sel}"
    # the embedded renderer supplies the rest of the ebiten.Game method set
    for m in ("Draw", "Layout", "SaveImage", "IsCompleted", "GetRenderDuration", "Update"):
        assert m in methods["BucketRenderer"], m
    assert re.search(r"func \(g \*GPUBucketRenderer\) Update\(\) error", src)
    assert re.search(r"func NewGPUBucketRenderer\(camera \*Camera, world Hittable, bucketSize int, numWorkers int\)",
                     src)


@pytest.mark.skipif(not os.path.isdir(REFERENCE_RT), reason="reference tree not present")
def test_no_undefined_functions():
    types, funcs, methods = _ref_decls()
    ours = ""
    for fn in sorted(os.listdir(RT_DIR)):
        ours += _read(os.path.join(RT_DIR, fn))
    code = re.sub(r"//.*", "", ours)
    code = re.sub(r'"(?:[^"\\]|\\.)*"', '""', code)
    defined = set(re.findall(r"^func (?:\([^)]*\) )?(\w+)\(", code, re.M))
    rtgpu_src = re.sub(r"//.*", "", _read(RTGPU_GO))
    rtgpu_exported = set(re.findall(r"^func (?:\([^)]*\) )?([A-Z]\w*)\(", rtgpu_src, re.M))
    rtgpu_exported |= set(re.findall(r"^type ([A-Z]\w*) ", rtgpu_src, re.M))
    rtgpu_exported |= set(re.findall(r"^\s*([A-Z]\w*)\s+(?:int32\s+)?=", rtgpu_src, re.M))
    std = {"fmt": {"Sprintf", "Fprintf", "Errorf"}, "math": {"Tan"}, "unsafe": {"Slice", "Pointer", "Sizeof"},
           "time": {"Now", "Since", "Duration", "Millisecond"}, "os": {"Getenv"}}
    for pkg, name in set(re.findall(r"\b(\w+)\.([A-Z]\w*)\b", code)):
        if pkg == "rtgpu":
            assert name in rtgpu_exported, f"rtgpu.{name} undefined"
        elif pkg in std:
            if name not in ("Stderr",):
                assert name in std[pkg], f"{pkg}.{name} not expected"
    # bare calls: ours, the reference package's, builtins or a local closure
    for name in set(re.findall(r"(?<![.\w])([A-Za-z_]\w*)\(", code)):
        assert (name in defined or name in funcs or name in GO_BUILTINS or name in types
                or name in ("errGPUUnsupported",)), f"call to undefined {name}"
    # method calls on receivers we own
    for name in set(re.findall(r"\b[fg]\.(\w+)\(", code)):
        assert name in defined or name in methods.get("BucketRenderer", set()), f"method {name} undefined"
