"""Restatement of the reference's calc_stepinfo (tools/general.py:46-61) -- TEST INFRASTRUCTURE.
Pure Python over lists, same expressions and the same None / exception behaviour."""


def calc_stepinfo(ys, y_base, error_band=0.05, ts=None):
    overshoot = ((max(ys) if y_base > 0 else min(ys)) - y_base) / y_base * 100 if y_base != 0 else None
    try:
        tr = ts[next(i for i in range(0, len(ys) - 1)
                     if (ys[i] - ys[0]) / (y_base - ys[0]) >= (1 - error_band))] - ts[0] if ts else None
    except StopIteration:
        tr = None
    try:
        tp = ts[next(len(ys) - i for i in range(1, len(ys) + 1)
                     if ((ys[len(ys) - i] - ys[0]) / (y_base - ys[0]) <= 1 - error_band
                         or (ys[len(ys) - i] - ys[0]) / (y_base - ys[0]) >= 1 + error_band))] - ts[0] if ts else None
    except StopIteration:
        tp = None
    return {"overshoot": overshoot, "settling_time": tp, "rise_time": tr, "static_error": abs(ys[-1] - y_base)}
