"""Diagnostics (not a test): the dependency bound of frame-pipelined
launches, simulated on the host from the real records (no GPU).

Each picture's deblocking chain is modelled as T(r, c) = max(T(r, c-1) +
period, T(r-1, c) + lag, ready(r, c) + period) with the in-situ period and
row lag of a one-step launch (tools/prof_chain.py: 2.25 us, 1.62 us), where
ready(r, c) is when MB (r, c)'s reference lines in the pictures of earlier
steps of the launch are final, under three rules:
  none     no wait (the H264MI_STUDY_NODEP bound: output not valid)
  row      rows 0..R+1 of the producer complete (the round-4 row tags)
  column   rows R_lo..R_hi through MB column X (+1 for the store lag) and row
           R_hi + 1 through X (recon_kernels.hip dep_wait)
  picture  the whole producer picture (one release per picture)
R_lo, R_hi, X are the lines of each MB's MC windows (mc_issue's geometry).
Prints the launch time per rule for SIM_P steps of SIM_S streams."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

PER = float(os.environ.get("SIM_PERIOD", "2.25"))
LAG = float(os.environ.get("SIM_LAG", "1.62"))
P = int(os.environ.get("SIM_P", "3"))
S = int(os.environ.get("SIM_S", "8"))
K0 = int(os.environ.get("SIM_K0", "6"))
DT = np.dtype([("type", "u1"), ("x", "u1", 15), ("i4", "<u2", 4), ("ref", "u1", 4), ("mv", "<i2", (16, 2)),
               ("slice", "<u2"), ("refidx", "<u2")])
BX = np.array([0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3])
BY = np.array([0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3])


def needs(rec, w, h):
    """per MB, per 4x4 block: ref slot, R_lo, R_hi, X (luma and chroma merged)"""
    W16, H16, CW, CH = w * 16, h * 16, w * 8, h * 8
    mb = np.arange(w * h)
    mbx, mby = (mb % w)[:, None], (mb // w)[:, None]
    mvx, mvy = rec["mv"][:, :, 0].astype(int), rec["mv"][:, :, 1].astype(int)
    x0 = np.clip((mbx * 16 + BX * 4 + (mvx >> 2) - 2) & ~3, 0, W16 - 12)
    y0 = mby * 16 + BY * 4 + (mvy >> 2) - 2
    lrlo, lrhi = np.clip(y0, 0, H16 - 1) >> 4, np.clip(y0 + 8, 0, H16 - 1) >> 4
    lx = np.minimum((x0 + 11) | 127, W16 - 1) >> 4
    cx0 = np.clip((mbx * 8 + BX * 2 + (mvx >> 3)) & ~3, 0, CW - 8)
    cy0 = mby * 8 + BY * 2 + (mvy >> 3)
    crlo, crhi = np.clip(cy0, 0, CH - 1) >> 3, np.clip(cy0 + 2, 0, CH - 1) >> 3
    cx = np.minimum((cx0 + 7) | 127, CW - 1) >> 3
    slot = np.repeat(rec["ref"], 4, axis=1)
    return slot, np.minimum(lrlo, crlo), np.maximum(lrhi, crhi), np.maximum(lx, cx)


def chain(w, h, ready):
    T = np.zeros((h, w))
    for r in range(h):
        for c in range(w):
            t = ready[r, c]
            if c:
                t = max(t, T[r, c - 1])
            if r:
                t = max(t, T[r - 1, c] + LAG - PER)
            T[r, c] = t + PER
    return T


def main():
    seeds = [100 + i for i in range(S)]
    ov = dict(kv.split("=") for kv in os.environ.get("SIM_GEN", "").split(",") if kv)
    _, caps = bench.prepare(3, seeds, K0 + P, {k: int(v) for k, v in ov.items()})
    w, h = caps[0].w_mbs, caps[0].h_mbs
    out = {}
    for rule in ("none", "row", "column", "picture"):
        ends = []
        for cap in caps:
            Ts, slots = [], []
            for j in range(P):
                k = K0 + j
                rec = np.frombuffer(cap.records_bytes(k), dtype=DT)
                ready = np.zeros((h, w))
                if j and rule != "none":
                    slot, rlo, rhi, X = needs(rec, w, h)
                    inter = rec["type"] <= 1
                    for jj in range(j):
                        Tp = Ts[jj]
                        hit = inter[:, None] & (slot == slots[jj])
                        if not hit.any():
                            continue
                        if rule == "picture":
                            # the whole producer picture complete
                            t = np.where(hit, Tp[h - 1, w - 1], 0.0)
                        elif rule == "row":
                            # rows 0..R_hi+1 complete: the last of them is the latest
                            rr = np.minimum(rhi + 1, h - 1)
                            t = np.where(hit, Tp[rr, w - 1], 0.0)
                        else:
                            xa = np.minimum(X + 1, w - 1)
                            t = np.maximum(Tp[rhi, xa], Tp[rlo, xa])
                            t = np.maximum(t, np.where(rhi + 1 < h, Tp[np.minimum(rhi + 1, h - 1), X], 0.0))
                            t = np.where(hit, t + 2 * PER, 0.0)      # store + publish lag
                        ready = np.maximum(ready, t.max(axis=1).reshape(h, w))
                T = chain(w, h, ready)
                Ts.append(T)
                slots.append(cap.pictures[k].cur_slot)
            ends.append(max(T[h - 1, w - 1] for T in Ts))
        out[rule] = np.mean(ends)
        print(f"{rule:7s} launch of {P} steps: {out[rule]:7.1f} us = {out[rule] / P:6.1f} per step (mean over {S} streams)")
    if os.environ.get("SIM_JSON"):
        # the data-dependent latency floor bench.py quotes beside its own
        # (roofline.latency.data_dependent_*), for the workload simulated here
        import json
        with open(os.environ["SIM_JSON"], "w") as f:
            json.dump({"workload": {"config": 3, "streams": S, "steps_per_launch": P, "pictures": [K0, K0 + P - 1],
                                    "gen_overrides": ov},
                       "period_us": PER, "lag_us": LAG,
                       "launch_us": {k: round(v, 1) for k, v in out.items()},
                       "source": "tools/dep_sim.py (SIM_PERIOD / SIM_LAG: the lone-wave costs of profiles/ubench.json)"},
                      f, indent=1)


if __name__ == "__main__":
    main()
