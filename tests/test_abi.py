"""The Rust binding crate (integration/rust/novelpoly-mi355x) against the C
header: the image has no Rust toolchain, so this checks what a compile would
catch first -- every entry point of include/novelpoly.h is declared in
src/sys.rs with the same number of parameters, nothing extra, and the status
constants agree with the header's enum (errors.rs:4-28 order)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(ROOT, "integration", "rust", "novelpoly-mi355x")


def _params(arglist):
    arglist = arglist.strip()
    if arglist in ("", "void"):
        return 0
    depth, n = 0, 1
    for ch in arglist:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        elif ch == "," and depth == 0:
            n += 1
    return n - (1 if arglist.rstrip().endswith(",") else 0)


def header_functions():
    src = open(os.path.join(ROOT, "include", "novelpoly.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(np_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        out[m.group(1)] = _params(m.group(2))
    return out


def rust_functions():
    src = open(os.path.join(CRATE, "src", "sys.rs")).read()
    src = re.sub(r"//[^\n]*", "", src)
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (np_[a-z0-9_]+)\s*\((.*?)\)\s*(?:->\s*[^;]+)?;", block, flags=re.S):
        out[m.group(1)] = _params(m.group(2))
    return out


def test_sys_rs_declares_every_header_function():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 30
    assert sorted(h) == sorted(r), (sorted(set(h) - set(r)), sorted(set(r) - set(h)))
    bad = {n: (h[n], r[n]) for n in h if h[n] != r[n]}
    assert not bad, bad


def test_status_constants_match_header():
    hdr = open(os.path.join(ROOT, "include", "novelpoly.h")).read()
    want = dict((k, int(v)) for k, v in re.findall(r"\b(NP_[A-Z0-9_]+)\s*=\s*(\d+)", hdr))
    rs = open(os.path.join(CRATE, "src", "sys.rs")).read()
    got = dict((k, int(v)) for k, v in re.findall(r"pub const (NP_[A-Z0-9_]+): c_int = (\d+);", rs))
    assert got == want


def test_error_mapping_covers_reference_variants():
    """lib.rs maps codes 1..8 onto the reference Error variants with their
    fields (errors.rs:4-28: WantedShardCountTooLow(usize) etc.)."""
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    for variant in ("WantedShardCountTooHigh(d[0])", "WantedShardCountTooLow(d[0])",
                    "WantedPayloadShardCountTooLow(d[0])", "PayloadSizeIsZero",
                    "NeedMoreShards { have: d[0], min: d[1], all: d[2] }",
                    "ParamterMustBePowerOf2 { n: d[0], k: d[1] }",
                    "InconsistentShardLengths { first: d[0], other: d[1] }", "EmptyShard"):
        assert "Error::" + variant in lib, variant
