"""Host-side Storage (b747_rl_ctrl_amd/storage.py) against the reference's semantics
(tools/general.py:315-379): record / clear / set_suffix / merge, unit labels of save(), CSV/npz output."""
import math
import os

import numpy as np
import pytest

from b747_rl_ctrl_amd.storage import STORAGE_COLUMNS, Storage, get_label_unit, place_unit


def test_label_units_follow_the_first_matching_prefix():
    # tools/general.py:130-144 in dict order: 'h' before 'U' ... 't' last
    assert get_label_unit("hzh") == "[м]" and get_label_unit("U_com") == "[В]" and get_label_unit("U_RL") == "[В]"
    assert get_label_unit("vartheta_ref") == "[град]" and get_label_unit("Vx") == "[м/с]"
    assert get_label_unit("wz") == "[1/с]" and get_label_unit("t") == "[с]" and get_label_unit("rew") == "[-]"
    assert get_label_unit("deltaz") == "[град]" and get_label_unit("x") == "[м]" and get_label_unit("Q") is None
    assert place_unit("vartheta__СС ПИД") == "vartheta, [град]__СС ПИД"
    assert place_unit("t") == "t, [с]" and place_unit("Q") == "Q"


def test_record_suffix_merge_clear():
    a, b = Storage(), Storage()
    for t in range(3):
        a.record("t", t * 0.01)
        a.record("vartheta", float(t))
        b.record("t", t * 0.01)
        b.record("vartheta", 2.0 * t)
    a.set_suffix("PID")
    a.merge(b, "model")
    assert list(a.storage) == ["t__PID", "vartheta__PID", "t__model", "vartheta__model"]
    assert a.storage["vartheta__model"] == [0.0, 2.0, 4.0]
    a.clear("t__model")
    assert "t__model" not in a.storage
    a.clear_all()
    assert a.storage == {}
    with pytest.raises(ValueError):
        a.save("x.csv")


def test_save_writes_unit_labelled_csv_and_npz(tmp_path):
    s = Storage()
    for t in range(4):
        for name in STORAGE_COLUMNS:
            s.record(name, t + 0.5 if name != "t" else t * 0.01)
    path = s.save(str(tmp_path / "sub" / "data.csv"), base="t")
    assert path.endswith(".csv") and os.path.exists(path)
    import pandas as pd
    df = pd.read_csv(path, index_col=0)
    assert df.index.name == "t, [с]" and "vartheta, [град]" in df.columns and "hzh, [м]" in df.columns
    assert np.allclose(df["U_RL, [В]"].to_numpy(), [0.5, 1.5, 2.5, 3.5])
    p2 = s.save(str(tmp_path / "data.npz"))
    z = np.load(p2)
    assert set(z.files) == set(STORAGE_COLUMNS) and z["t"][-1] == 0.03


def _read_xlsx(path):
    """every part parsed (well-formed XML), sheet "data" as rows of {column letter: text}"""
    import re
    import xml.etree.ElementTree as ET
    import zipfile
    ns = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
    with zipfile.ZipFile(path) as z:
        parts = {n: ET.fromstring(z.read(n)) for n in z.namelist()}
    wb = parts["xl/workbook.xml"]
    assert [e.get("name") for e in wb.iter("{%s}sheet" % ns["m"])] == ["data"]
    rows = []
    for row in parts["xl/worksheets/sheet1.xml"].iter("{%s}row" % ns["m"]):
        cells = {}
        for c in row.findall("m:c", ns):
            col = re.match(r"[A-Z]+", c.get("r")).group(0)
            v = c.find("m:v", ns)
            cells[col] = "".join(t.text or "" for t in c.iter("{%s}t" % ns["m"])) if c.get("t") == "inlineStr" \
                else v.text
        rows.append(cells)
    return parts, rows


def test_save_xlsx_writes_the_reference_workbook(tmp_path):
    """Storage.save("x.xlsx") -> write_dataframe's workbook (tools/general.py:230-312) and its "_big" copy
    (:366-369), written without openpyxl (b747_rl_ctrl_amd/xlsx.py)"""
    s, rng = Storage(), np.random.default_rng(3)
    vals = {name: rng.normal(size=6) * 10.0 ** rng.integers(-8, 5) for name in STORAGE_COLUMNS}
    vals["t"] = np.arange(6) * 0.01
    for t in range(6):
        for name in STORAGE_COLUMNS:
            s.record(name, float(vals[name][t]))
    path = s.save(str(tmp_path / "out" / "run.xlsx"), base="t")
    assert path.endswith("run.xlsx") and os.path.exists(tmp_path / "out" / "run_big.xlsx")
    parts, rows = _read_xlsx(path)
    header = rows[0]
    assert header["A"] == "t, [с]"
    labels = [header[k] for k in sorted(header, key=lambda c: (len(c), c)) if k != "A"]
    assert labels == [place_unit(c) for c in STORAGE_COLUMNS if c != "t"]
    for j, name in enumerate([c for c in STORAGE_COLUMNS if c != "t"]):
        col = chr(ord("B") + j)
        assert [float(r[col]) for r in rows[1:]] == list(vals[name])          # exact: repr round trip
    assert [float(r["A"]) for r in rows[1:]] == list(vals["t"])
    charts = sorted(n for n in parts if n.startswith("xl/charts/"))
    groups = [c for c in STORAGE_COLUMNS if c != "t"]                          # one chart per group
    assert len(charts) == len(groups)
    c_ns = "{http://schemas.openxmlformats.org/drawingml/2006/chart}"
    series = {n: [f.text for f in parts[n].iter(c_ns + "f")] for n in charts}
    th = next(n for n, fs in series.items() if any("$L$" in f for f in fs))   # vartheta is column L
    assert len(series[th]) == 4                                                # + vartheta_ref (x and y refs)
    assert all(f.startswith("'data'!$") and f.endswith("$7") for fs in series.values() for f in fs)
    _, big_rows = _read_xlsx(str(tmp_path / "out" / "run_big.xlsx"))
    assert big_rows == rows
    with __import__("zipfile").ZipFile(str(tmp_path / "out" / "run_big.xlsx")) as z:
        assert 'sz="4000"' in z.read(charts[0]).decode()


def test_plot_to_file(tmp_path):
    s = Storage()
    for t in range(5):
        s.record("t", t * 0.01)
        s.record("vartheta", math.sin(t))
    p = str(tmp_path / "p.png")
    s.plot(["vartheta"], "t", "t, [с]", "ϑ, [град]", path=p)
    assert os.path.getsize(p) > 0


def test_xlsx_package_matches_the_reference_workbook(tmp_path):
    """The writer's package against the reference's own openpyxl workbook (tests/golden/xlsx_package.json from
    tensorboard.xlsx): the same part kinds, content types and relationship types, the optional theme part aside"""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_xlsx_fixture import structure
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "xlsx_package.json")))
    s = Storage()
    for t in range(4):
        s.record("t", t * 0.01)
        s.record("vartheta", math.sin(t))
        s.record("deltaz", math.cos(t))
    got = structure(s.save(str(tmp_path / "run.xlsx"), base="t"))
    theme = "xl/theme/themeN.xml"
    assert got["parts"] == [p for p in ref["parts"] if p != theme]
    assert got["content_types"] == {k: v for k, v in ref["content_types"].items() if k != theme}
    wb = "xl/_rels/workbook.xml.rels"
    assert got["rels"] == {**ref["rels"], wb: [r for r in ref["rels"][wb] if not r.endswith("/theme")]}
    assert got["sheet"] == ref["sheet"]
