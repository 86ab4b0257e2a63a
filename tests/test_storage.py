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
    path = s.save(str(tmp_path / "sub" / "data.xlsx"), base="t")   # no openpyxl here: CSV next to it
    assert path.endswith(".csv") and os.path.exists(path)
    import pandas as pd
    df = pd.read_csv(path, index_col=0)
    assert df.index.name == "t, [с]" and "vartheta, [град]" in df.columns and "hzh, [м]" in df.columns
    assert np.allclose(df["U_RL, [В]"].to_numpy(), [0.5, 1.5, 2.5, 3.5])
    p2 = s.save(str(tmp_path / "data.npz"))
    z = np.load(p2)
    assert set(z.files) == set(STORAGE_COLUMNS) and z["t"][-1] == 0.03


def test_plot_to_file(tmp_path):
    s = Storage()
    for t in range(5):
        s.record("t", t * 0.01)
        s.record("vartheta", math.sin(t))
    p = str(tmp_path / "p.png")
    s.plot(["vartheta"], "t", "t, [с]", "ϑ, [град]", path=p)
    assert os.path.getsize(p) > 0
