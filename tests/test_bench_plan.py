"""bench.py's launch plans on the CPU (dry engine): the GOP-staggered plan
with one and with two steps per launch (frame-pipelined launches, verdict
r03 #8).  Every stream must see its pictures in cyclic decode order, the
pre-roll must bring stream s to its phase, a two-step launch must pair
pictures (k, k+1) of every stream with k even, and the descriptor table must
hold exactly the plan's pictures."""
import bench
from broadway_amd import gen
from broadway_amd.engine import Capture


def _walk(launches, S):
    """Per stream, the picture sequence the plan decodes."""
    seq = [[] for _ in range(S)]
    for launch in launches:
        for step in launch:
            for s, k in enumerate(step):
                seq[s].append(k)
    return seq


def test_gop_phases_whole_launches():
    assert bench.gop_phases(8, 60) == [0, 7, 15, 22, 30, 37, 45, 52]
    # two steps per launch: odd phases (a stream's IDR is the second picture
    # of its launch), or even ones with offset 0
    assert bench.gop_phases(8, 60, 2) == [1, 7, 15, 23, 31, 37, 45, 53]
    assert bench.gop_phases(8, 60, 2, 0) == [0, 6, 14, 22, 30, 36, 44, 52]
    assert all(p % 2 == 1 for p in bench.gop_phases(5, 60, 2))


def test_launch_plan_pipe2_cyclic():
    N, S, W, K = 60, 8, 4, 56
    ph = bench.gop_phases(S, N, 2)
    launches, R = bench.launch_plan(N, S, W, K, ph, None, 2)
    assert R == max(ph)
    assert all(len(x) == 1 for x in launches[:R]) and all(len(x) == 2 for x in launches[R:])
    for launch in launches[R:]:
        for s in range(S):
            a, b = launch[0][s], launch[1][s]
            assert a % 2 == 1 and b == (a + 1) % N          # odd phases: (k, k + 1), k odd; (59, 0) wraps
    seq = _walk(launches, S)
    for s in range(S):
        main = seq[s][R:]
        assert main == [(v + ph[s]) % N for v in range(W + K)]
        # pre-roll: repeats of the IDR, then pictures 0 .. phase-1 in order
        pre = [k for k in seq[s][:R]]
        tail = pre[R - ph[s]:] if ph[s] else []
        assert tail == list(range(ph[s])) and all(k == 0 for k in pre[:R - ph[s]])


def _caps(n=3, frames=12):
    streams = [gen.generate(2, 90 + i, nframes=frames, w_mbs=13, h_mbs=7, crop_bottom=0, slices=2, gop=frames)
               for i in range(n)]
    return [Capture(s) for s in streams]


def test_device_run_pipe2_odd_phases_never_split():
    """Odd phases: every IDR is the second picture of its launch, paired with
    the stream's previous GOP's last picture (no dependency), so every main
    launch has two steps."""
    caps = _caps()
    S, N = len(caps), 12
    ph = bench.gop_phases(S, N, 2)
    run = bench.DeviceRun(None, caps, 2, 8, 2, dry=True, phases=ph)
    assert run.P == 2
    main = run.launches[run.n_pre:]
    assert all(len(x) == 2 for x in main) and any(run.holds_idr(x) for x in main)
    assert not any(run.holds_idr(x[:1]) for x in main)
    seq = _walk(main, S)
    assert all(seq[s] == [(v + ph[s]) % N for v in range(10)] for s in range(S))
    run.free()


def test_device_run_pipe2_gop_plan_descriptors():
    caps = _caps()
    S, N = len(caps), 12
    ph = bench.gop_phases(S, N, 2, 0)
    run = bench.DeviceRun(None, caps, 2, 8, 2, dry=True, phases=ph)
    assert run.P == 2
    # launches holding an IDR run one step at a time, the others two
    main = run.launches[run.n_pre:]
    assert all(not run.holds_idr(x) for x in main if len(x) == 2)
    singles = [j for j, x in enumerate(main) if len(x) == 1]
    assert len(singles) % 2 == 0 and singles
    for j in singles[::2]:
        assert len(main[j + 1]) == 1 and run.holds_idr(main[j] + main[j + 1])
    assert sum(len(x) for x in main) == 10
    assert sum(len(x) for x in main[:run.n_warm - run.n_pre]) == 2
    seq = _walk(main, S)
    assert all(seq[s] == [(v + ph[s]) % N for v in range(10)] for s in range(S))
    # the table, launch by launch, is the plan's pictures step-major
    assert run.desc_off[-1] == sum(len(x) for x in run.launches) * S * 32
    # a two-step launch's pictures write distinct slots
    for launch in [x for x in main if len(x) == 2]:
        for s in range(S):
            assert run.slot_of[launch[0][s]][s] != run.slot_of[launch[1][s]][s]
    for i in range(len(run.launches)):
        run.launch(i)
    assert run.eng.launches == len(run.launches)
    # the P-only window of bench.main: phases [2]*S, whole launches
    run.set_plan(2, 6, [2] * S)
    assert all(not run.is_i[k][s] for s, k in run.timed_pictures())
    run.free()


def test_device_run_odd_warmup_and_steps():
    """The driver's window (odd warmup, any step count): warmup % 2 single
    steps first, then pairs starting at the timed window's first step, a
    single last when the steps are odd; phases of the parity that makes every
    IDR a pair's second picture."""
    caps = _caps()
    S, N, W, K = len(caps), 12, 3, 7
    ph = bench.gop_phases(S, N, 2, (W + 1) % 2)
    run = bench.DeviceRun(None, caps, W, K, 2, dry=True, phases=ph)
    assert run.P == 2
    main = run.launches[run.n_pre:]
    assert [len(x) for x in main] == [1, 2, 2, 2, 2, 1]
    assert run.n_warm - run.n_pre == 2                      # the single + one pair: 3 warmup steps
    assert not any(run.holds_idr(x[:1]) for x in main if len(x) == 2)
    seq = _walk(main, S)
    assert all(seq[s] == [(v + ph[s]) % N for v in range(W + K)] for s in range(S))
    run.free()


def test_device_run_pipe3_idr_last():
    """Three steps per launch: physical slots renamed onto enough slots that
    every launch -- the cyclic one across the GOP wrap included -- meets the
    batch contract, every IDR the last picture of its launch, the driver's
    odd warmup as leading single steps."""
    caps = _caps()
    S, N = len(caps), 12
    for W, K in ((3, 9), (4, 8), (5, 7)):
        ph = bench.gop_phases(S, N, 3, warmup=W)
        run = bench.DeviceRun(None, caps, W, K, 3, dry=True, phases=ph)
        assert run.P == 3 and run.nslots >= 3
        main = run.launches[run.n_pre:]
        rest = W + K - W % 3
        assert [len(x) for x in main] == [1] * (W % 3) + [3] * (rest // 3) + ([rest % 3] if rest % 3 else [])
        assert any(run.holds_idr(x) for x in main) and not any(run.holds_idr(x[:-1]) for x in main)
        assert bench.pairs_ok(run.recs_h, run.pics_h, S, run.nmbs, N, 3, (W + ph[0]) % 3)
        seq = _walk(main, S)
        assert all(seq[s] == [(v + ph[s]) % N for v in range(W + K)] for s in range(S))
        for launch in main:
            for s in range(S):
                slots = [run.slot_of[st[s]][s] for st in launch]
                assert len(set(slots)) == len(slots)
        run.free()


def test_latency_floors_from_committed_profiles():
    """roofline.latency: the lone-wave picture floor (profiles/ubench.json)
    and the data-dependent launch floor (profiles/dep_floor.json), the latter
    only for the workload it was simulated on."""
    ub = bench.load_ubench()
    assert ub is not None
    dep = bench.load_dep_floor(3, 8, 3, "")
    assert dep is not None and dep["launch_us"]["none"] <= dep["launch_us"]["row"]
    assert bench.load_dep_floor(4, 1, 3, "") is None and bench.load_dep_floor(3, 8, 3, "offpic_pct=0") is None
    lf = bench.latency_floor(120, 68, 3, ub, 883.0, dep)
    assert abs(lf["picture_floor_us"] - (120 * ub["vh_us"] + 67 * (ub["patch_us"] + ub["hop_same_xcd_us"]))) < 0.01
    assert lf["launch_floor_us"] < lf["data_dependent_launch_floor_us"] < 883.0
    assert abs(lf["data_dependent_frac"] - dep["launch_us"]["row"] / 883.0) < 1e-3
    assert bench.latency_floor(120, 68, 3, ub, 883.0)["data_dependent_frac"] is None
