"""The model constants: include/b747_tables.h == gen/params.json == the DLL's .data bytes."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DLL = "/root/reference/core/model_simple_win64.dll"
PARAMS = os.path.join(ROOT, "gen", "params.json")


def test_params_json_matches_reference_dll():
    if not os.path.exists(DLL):
        pytest.skip("reference DLL not mounted (GPU box)")
    sys.path.insert(0, os.path.join(ROOT, "gen"))
    import extract_params
    fresh = extract_params.extract(DLL)
    stored = json.load(open(PARAMS, encoding="utf-8"))
    assert fresh == stored


def test_header_is_generated_from_params():
    hdr = open(os.path.join(ROOT, "include", "b747_tables.h")).read()
    P = json.load(open(PARAMS, encoding="utf-8"))
    arrays = dict((m.group(1), [float(x) for x in m.group(2).split(",")])
                  for m in re.finditer(r"double (B747_\w+)\[\d+\] = \{([^}]*)\}", hdr))
    F = "model_simple/B747/Расчет а//д сил в скоростной СК/"
    M = "model_simple/B747/Расчет а//д моментов в связной СК/"
    bp = P["block_parameters"]
    assert arrays["B747_CXA_TBL"] == bp[F + "CXa.Table"]["value"]
    assert arrays["B747_CYA_BP1"] == bp[F + "CYa.BreakpointsForDimension2"]["value"]
    assert arrays["B747_DCM_TBL"] == bp[M + "dCm//ddeltaz_table.Table"]["value"]
    assert arrays["B747_MZ_BP1"] == bp[M + "mz_table.BreakpointsForDimension2"]["value"]
    assert arrays["B747_KA_TBL"] == bp[M + "Kalpha_table.Table"]["value"]
    assert arrays["B747_DEF_PID_SS"] == P["model_parameters"]["PID_SS"]["value"]
    # every breakpoint vector strictly increasing (required by the branch-free index search)
    for k, v in arrays.items():
        if "_BP" in k:
            assert all(a < b for a, b in zip(v, v[1:])), k
    # SURVEY A.7 spot values
    assert "#define B747_DEF_IZ (67300000.0)" in hdr and "#define B747_DEF_P (275000.0)" in hdr
    assert "#define B747_DELAY_INIT (-0.000171374)" in hdr


def test_header_regeneration_is_stable(tmp_path):
    """Regenerate into a temp path (never rewrite the tracked header: its mtime is a build
    dependency of libb747.so) and compare."""
    import subprocess
    hdr = os.path.join(ROOT, "include", "b747_tables.h")
    before, mtime = open(hdr).read(), os.path.getmtime(hdr)
    out = tmp_path / "b747_tables.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "gen", "gen_tables.py"), str(out)], check=True,
                   capture_output=True)
    assert out.read_text() == before
    assert os.path.getmtime(hdr) == mtime
