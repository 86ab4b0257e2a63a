"""Extract the reference's own recorded closed-loop test results into tests/golden/tb_transfer_first_log.json
(TEST INFRASTRUCTURE; run once in the build container, where /root/reference exists).

/root/reference/tensorboard.xlsx (exported by tools/tb_convert.py:3-60) holds the SB3 training curves of the 18
runs main.py:100-110 trains: obs PID_LIKE / SPEED_MODE x ctrl mode DIRECT / ADD_DIRECT / ADD_PROC x reset mode
CONST / HYBRID / OSCILLATING.  Its `transfer_custom/{overshoot,quality,settling_time}` columns are written by
ControlTestCallback.calc_stepinfo (neural/callbacks.py:60-100): the test env of main.py:57-72 (tk 20 s,
sample_time 0.05, no disturbance), state0 [0, 11000, 250, 0, 0, 0] (main.py:124), references +-5 and +-10 deg
(main.py:116), the deterministic policy, a fresh DLL per reference -- i.e. numbers the reference's DLL produced.
The first log point (timestep 8192 = SB3's default n_steps 2048 x the 4 worker envs of neural/agent.py:63-81,
since neural/setups.py:29 keys PPO by the string 'PPO' and ControllerAgent looks it up by class, agent.py:48-53)
is taken with the policy still at its initial weights, so it is PID (ADD_* modes) or open loop (DIRECT) plus
the initial policy's tiny actions -- a state our oracle can reproduce (tests/tb_transfer.py).  The same row's
rollout/ep_rew_mean, ep_len_mean are SB3's statistics over the 20 training episodes (4 workers x 5 x 400 steps)
finished by then: the train env (main.py:41-55, random resets) under the initial stochastic policy (std 1).
The train/* columns start one row later (timestep 16384): PPO.train's statistics of the first update over that
rollout, dumped with the next rollout's row ("train" in the fixture).

tests/golden/tb_curves.json keeps every row of the episode-reward, transfer and train/* curves (62 log points per
run) for the full training replay (tests/tb_training.py).

The workbook is read as data: zipfile + xml.etree on the sheet and shared-string XML, no workbook code.
  python tests/golden/make_tb_fixture.py [path/to/tensorboard.xlsx]"""
import json
import os
import re
import sys
import xml.etree.ElementTree as ET
import zipfile

HERE = os.path.dirname(os.path.abspath(__file__))
NS = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}
OUT = os.path.join(HERE, "tb_transfer_first_log.json")
CURVES = os.path.join(HERE, "tb_curves.json")
CURVE_TAGS = ("rollout/ep_rew_mean", "transfer_custom/settling_time", "transfer_custom/overshoot",
              "transfer_custom/quality", "train/approx_kl", "train/clip_fraction", "train/entropy_loss",
              "train/explained_variance", "train/loss", "train/policy_gradient_loss", "train/std", "train/value_loss")


def _text(el):
    return "".join(t.text or "" for t in el.iter(f"{{{NS['m']}}}t"))


def read_sheet(path):
    """[{column letter: cell text}] of sheet1, row by row"""
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        shared = []
        if "xl/sharedStrings.xml" in names:
            shared = [_text(si) for si in ET.fromstring(z.read("xl/sharedStrings.xml")).findall("m:si", NS)]
        root = ET.fromstring(z.read("xl/worksheets/sheet1.xml"))
    rows = []
    for row in root.iter(f"{{{NS['m']}}}row"):
        cells = {}
        for c in row.findall("m:c", NS):
            col = re.match(r"[A-Z]+", c.get("r")).group(0)
            v = c.find("m:v", NS)
            if c.get("t") == "s":
                cells[col] = shared[int(v.text)]
            elif c.get("t") == "inlineStr":
                cells[col] = _text(c)
            elif v is not None:
                cells[col] = v.text
        rows.append(cells)
    return rows


def main(path):
    rows = read_sheet(path)
    header, data = rows[0], rows[1:]
    runs = {}
    for col, name in header.items():
        t = re.match(r"train/(\w+)__(.+)$", name)
        if t:                                   # SB3's first PPO update, logged with the next rollout's row
            first = next(r for r in data if r.get(col))
            run = runs.setdefault(t.group(2), {})
            tr = run.setdefault("train", {"step": int(first["A"])})
            assert tr["step"] == int(first["A"])
            tr[t.group(1)] = float(first[col])
            continue
        m = re.match(r"(?:transfer_custom|rollout)/(overshoot|quality|settling_time|ep_rew_mean|ep_len_mean)__(.+)$",
                     name)
        if not m:
            continue
        first = next(r for r in data if r.get(col))
        run = runs.setdefault(m.group(2), {})
        run.setdefault("step", int(first["A"]))
        assert run["step"] == int(first["A"])
        run[m.group(1)] = float(first[col])
    assert len(runs) == 18, sorted(runs)
    doc = {"source": "tensorboard.xlsx sheet1, first row of every transfer_custom/* column "
                     "(ControlTestCallback.calc_stepinfo, neural/callbacks.py:60-100) and of rollout/ep_rew_mean, "
                     "rollout/ep_len_mean (SB3 episode statistics of the 20 training episodes finished by then); 'train': "
                     "the first row of every train/* column (SB3 PPO.train of the first update, timestep 16384)",
           "runs": {k: runs[k] for k in sorted(runs)}}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}: {len(runs)} runs")
    curves = {}
    for col, name in header.items():
        tag, _, run = name.partition("__")
        if tag in CURVE_TAGS:
            curves.setdefault(run, {})[tag] = [[int(r["A"]), float(r[col])] for r in data if r.get(col)]
    with open(CURVES, "w") as f:
        json.dump({"source": "tensorboard.xlsx sheet1: every row of the listed columns, [timestep, value]",
                   "runs": {k: curves[k] for k in sorted(curves)}}, f, separators=(",", ":"))
        f.write("\n")
    print(f"wrote {CURVES}: {len(curves)} runs x {len(CURVE_TAGS)} curves")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tensorboard.xlsx")
