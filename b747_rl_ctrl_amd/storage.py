"""Storage -- the reference's step recorder (tools/general.py:315-379) and its batched GPU form.

`Storage` is the reference class with the same methods and semantics: `record(name, value)` appends
to a named column, `clear` / `clear_all`, `set_suffix` / `merge` rename columns as
`<name>__<suffix>` (tools/general.py:29 model_separator), `plot` draws columns (optionally against a
base column), and `save` writes the table with each column's unit appended to its label
(`place_unit`: "t, [с]", "vartheta, [град]", "vartheta__model, [град]"...).  `save("x.xlsx")` writes the
reference's workbook -- sheet "data" with one scatter chart per column group -- and its "x_big.xlsx" copy
through `b747_rl_ctrl_amd.xlsx` (openpyxl, which the reference uses, is not installed here); ".csv" and ".npz"
targets are written directly.

`BatchStorage` is `Controller.storage` for N environments at once.  `Controller._post_step`
(core/controller.py:209-228) appends, after EVERY DLL step, the columns
    t, U_com, U_PID, deltaz [deg], hzh, vartheta_ref [deg], U_RL (when an action was given),
    x, y, Vx, Vy, vartheta [deg], wz                (the NaN-scrubbed state, core/model.py:200, 226)
Here one env step's kernel (signal recording on: b747_env_batch.sig and .rec_params) leaves the 31
exported signals of each of its DLL steps and the DLL parameters the step ran with on the device;
`record_step` turns them into those columns as ONE device tensor [n_sub, 13, N] per env step (no
host round trip), and `storage(i)` / `columns()` hand env i's table / all tables back.
"""
import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch

MODEL_SEPARATOR = "__"                 # tools/general.py:29
LABEL_UNITS = {                        # tools/general.py:130-144 (first matching prefix wins)
    "h": "м", "U": "В", "vartheta": "град", "alpha": "град", "wz": "1/с", "rew": "-", "deltaz": "град",
    "x": "м", "y": "м", "V": "м/с", "ax": "м/с^2", "ay": "м/с^2", "t": "с",
}
STORAGE_COLUMNS = ["t", "U_com", "U_PID", "deltaz", "hzh", "vartheta_ref", "U_RL",
                   "x", "y", "Vx", "Vy", "vartheta", "wz"]      # core/controller.py:213-227 record order
_DEG = 180 / math.pi


def get_label_unit(label: str) -> Optional[str]:
    """tools/general.py:176-180: the unit of the first LABEL_UNITS prefix of label, as "[unit]"."""
    for target, unit in LABEL_UNITS.items():
        if label[:len(target)] == target:
            return f"[{unit}]"
    return None


def place_unit(label: str) -> str:
    """Storage.save's column naming (tools/general.py:353-364): "<name>, [unit]" (the unit of the part
    before the model separator)."""
    if MODEL_SEPARATOR in label:
        parts = label.split(MODEL_SEPARATOR)
        unit = get_label_unit(parts[0])
        if unit:
            parts[0] = f"{parts[0]}, {unit}"
        return MODEL_SEPARATOR.join(parts)
    unit = get_label_unit(label)
    return f"{label}, {unit}" if unit else label


class Storage:
    """tools/general.py:315-379."""

    def __init__(self):
        self.storage: Dict[str, list] = {}

    def record(self, name, value):
        if name not in self.storage:
            self.storage[name] = []
        self.storage[name].append(value)

    def clear(self, name):
        del self.storage[name]

    def clear_all(self):
        self.storage = {}

    def plot(self, names, base: Optional[str] = None, xlabel=None, ylabel=None, path: Optional[str] = None):
        """Columns `names` against `base` (or their index); shown, or saved to `path` when given."""
        import matplotlib
        if path is not None:
            matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        if isinstance(names, str):
            names = [names]
        fig = plt.figure()
        for name in names:
            if base and base in self.storage:
                plt.plot(self.storage[base], self.storage[name], label=name)
            else:
                plt.plot(self.storage[name], label=name)
        plt.grid()
        plt.legend()
        if xlabel:
            plt.xlabel(xlabel)
        if ylabel:
            plt.ylabel(ylabel)
        if path is not None:
            fig.savefig(path)
            plt.close(fig)
        else:
            plt.show()

    def save(self, filename: str = "storage.xlsx", base: Optional[str] = None) -> str:
        """The table with units in the column labels, indexed by `base` when given; returns the path
        written (".xlsx": the reference's workbook with charts and its "_big" copy; ".csv"; ".npz")."""
        import pandas as pd
        if len(self.storage) == 0:
            raise ValueError("Невозможно сохранить хранилище: пустое хранилище")   # tools/general.py:349
        d = os.path.dirname(filename)
        if d:
            os.makedirs(d, exist_ok=True)
        data = pd.DataFrame.from_dict(self.storage, orient="columns")
        data.columns = [place_unit(c) for c in data.columns]
        if base and base in self.storage:
            data.set_index(place_unit(base), inplace=True)
        stem, ext = os.path.splitext(filename)
        if ext == ".npz":
            np.savez(filename, **{c: np.asarray(v, dtype=np.float64) for c, v in self.storage.items()})
            return filename
        if ext == ".xlsx":
            # write_dataframe (tools/general.py:230-312): sheet "data" + one scatter chart per column group, and
            # the "<stem>_big" copy with 40 pt text and 7 pt lines (Storage.save, :366-369); b747_rl_ctrl_amd.xlsx
            # writes the workbook itself (openpyxl is not installed here)
            from .xlsx import write_table
            cols = [str(c) for c in data.columns]
            vals = [data[c].tolist() for c in data.columns]
            name = "" if data.index.name is None else str(data.index.name)
            write_table(filename, name, data.index.tolist(), cols, vals)
            write_table(stem + "_big" + ext, name, data.index.tolist(), cols, vals, big=True)
            return filename
        data.to_csv(filename, index=True, header=True)
        return filename

    def set_suffix(self, suffix: str):
        self.storage = {f"{k}{MODEL_SEPARATOR}{suffix}": v for k, v in self.storage.items()}

    def merge(self, obj: "Storage", suffix: str):
        self.storage.update({f"{k}{MODEL_SEPARATOR}{suffix}": v for k, v in obj.storage.items()})


class BatchStorage:
    """Controller.storage for every env of a BatchControllerEnv (see the module docstring).

    Columns are kept on the device as float64 [T, N] (T = DLL steps recorded); `extra` columns
    (e.g. the agent test's "rew", neural/agent.py:240-244) are recorded once per env step with
    `record(name, values[N])` and repeated over the env step's DLL steps like the reference's
    _post_step does.

    Episodes: Controller.reset backs the storage up and clears it (core/controller.py:195-199), so the
    reference's storage only ever holds the current episode.  Here every env keeps a window into the
    recorded rows: an explicit reset (masked or not) or an auto-reset at done starts a new one, and
    `storage(i)` / `storage_backup(i)` return env i's current / previous episode.  `columns()` keeps every
    row since the last `clear_all()` (the batched agent test resets all envs together, so there it is the
    episode); `clear_all()` also releases the rows."""

    def __init__(self, env):
        self.env = env
        self.clear_all()

    def clear_all(self):
        self._steps: List[torch.Tensor] = []          # per env step: [n_sub, 13, N]
        self._has_action: List[bool] = []
        self._extra: Dict[str, List[torch.Tensor]] = {}
        self._rows = 0                                # DLL steps recorded = len(self)
        z = lambda: torch.zeros(self.env.n, dtype=torch.int64, device=self.env.device)
        self._start, self._prev = z(), z()            # env i: current episode = rows [_start, T), backup = [_prev, _start)

    def episode_reset(self, mask: Optional[torch.Tensor] = None):
        """A new episode for every env (mask None) or where mask is true: the current one becomes the
        backup (Controller.reset, core/controller.py:195-199).  Stays on the device (no host sync)."""
        t = torch.full_like(self._start, self._rows)
        if mask is None:
            self._prev, self._start = self._start, t
        else:
            m = mask.to(device=self._start.device, dtype=torch.bool).reshape(-1)
            self._prev = torch.where(m, self._start, self._prev)
            self._start = torch.where(m, t, self._start)

    def __len__(self):
        return self._rows

    def record_step(self, action_scaled: Optional[torch.Tensor]):
        """Append the columns of the env step that just ran (signal recording must be on)."""
        from .model import SIG
        env = self.env
        sig, par = env.sig, env.rec_params               # [n_sub, 31, N], [3, N]
        ns, n = sig.shape[0], sig.shape[2]
        out = torch.empty(ns, len(STORAGE_COLUMNS), n, dtype=torch.float64, device=sig.device)
        out[:, 0] = sig[:, SIG["sim_time"]]
        out[:, 1] = sig[:, SIG["U_com"]]
        out[:, 2] = sig[:, SIG["U_com_PID"]]
        # the reference's own roundings: `deltaz_real*180/pi` and `vartheta_ref*180/pi` evaluate (x*180)/pi,
        # the state's `v *= 180/pi` evaluates x*(180/pi) (core/controller.py:217-227)
        out[:, 3] = sig[:, SIG["deltaz_RP"]] * 180 / math.pi
        out[:, 4] = par[1]
        # Controller.vartheta_ref (core/controller.py:268-270): the CS PID's output signal when it is in
        # the loop, else the DLL parameter vartheta the step ran with
        use_ctrl = (env.flags & 2).bool()                                       # F_PID_CS
        out[:, 5] = torch.where(use_ctrl, sig[:, SIG["vartheta_zh"]], par[0]) * 180 / math.pi
        out[:, 6] = action_scaled.to(torch.float64) if action_scaled is not None else math.nan
        st = torch.nan_to_num(sig[:, SIG["state_x"]:SIG["state_x"] + 6])       # core/model.py:200
        out[:, 7:13] = st
        out[:, 11] *= _DEG                                                      # vartheta in degrees
        self._steps.append(out)
        self._has_action.append(action_scaled is not None)
        self._rows += ns

    def record(self, name: str, values):
        """An extra per-env column for the env step recorded last (e.g. 'rew')."""
        v = torch.as_tensor(values, dtype=torch.float64, device=self.env.device).reshape(-1)
        ns = int(self._steps[-1].shape[0]) if self._steps else 1
        self._extra.setdefault(name, []).append(v[None].expand(ns, -1))

    def columns(self) -> Dict[str, torch.Tensor]:
        """Every column as a device tensor [T, N] (U_RL only when every step had an action)."""
        if not self._steps:
            return {}
        allc = torch.cat(self._steps, 0)
        cols = {name: allc[:, j] for j, name in enumerate(STORAGE_COLUMNS)}
        if not all(self._has_action):
            del cols["U_RL"]
        out = {}
        for name, v in self._extra.items():                                     # recorded first, as the
            out[name] = torch.cat(v, 0)                                          # agent's wrapper does
        out.update(cols)
        return out

    def _window(self, i: int, lo: int, hi: int) -> Storage:
        s = Storage()
        for name, v in self.columns().items():
            s.storage[name] = v[lo:hi, i].cpu().numpy().tolist()
        return s

    def storage(self, i: int) -> Storage:
        """Env i's current episode as the reference's Storage (host lists of floats)."""
        return self._window(i, int(self._start[i]), self._rows)

    def storage_backup(self, i: int) -> Storage:
        """Env i's previous episode (Controller.storage_backup, core/controller.py:198)."""
        return self._window(i, int(self._prev[i]), int(self._start[i]))
