"""Streaming sliding-window encode (quic-fec-eps_amd/csrc/fec_swenc.hip; ctx tuning
"sw_stream" 1..5 = that many dwords per lane, 6 = chosen per symbol size) against the CPU oracle
(oracle/fec_oracle.c orc_sw_encode) and against the combine-job encode
("sw_stream" 0).  Bit-exact on bytes [0, S) of every repair.

The workgroup's slot shape (P passes x A accumulator slots) follows the
headers of each segment, so the cases cover: regular schedules (W a multiple of
the step, and not), the widest window (P > 1), steps longer than the window
(holes between windows), stream-start clipping, windows out of order and
repeated (large A P), empty windows (device headers clipped to nothing),
ragged last segments, and symbols wider than one column pass.
PARITY UNPINNED vs the fec branch (not mounted)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import fecgpu  # noqa: E402
import oracle as O  # noqa: E402
import np_oracle as N  # noqa: E402

pytestmark = pytest.mark.gpu
MODES = (0, 1, 2, 3, 4, 5, 6)   # 0 the combine-job encode; 3 / 5 fall back to a divisor of the row's dwords


@pytest.fixture(scope="module")
def ctxs():
    assert torch.cuda.is_available()
    O.build()
    out = {}
    for mode in MODES:
        c = fecgpu.Context()
        c.set_tuning("sw_stream", mode)
        out[mode] = c
    yield out
    for c in out.values():
        c.close()


def hdr_array(h):
    a = np.zeros(len(h), O.SW_REPAIR_DTYPE)
    for t, (fss, nss, key, dt) in enumerate(h):
        a[t]["fss"], a[t]["nss"], a[t]["key"], a[t]["dt"] = fss, nss, key, dt
    return a


def stream(nsrc, L, stride, seed):
    rng = np.random.default_rng(seed)
    src = np.zeros((nsrc, stride), np.uint8)
    src[:, :L] = rng.integers(0, 256, (nsrc, L), dtype=np.uint8)
    return src


def gpu_encode(ctx, src, hdr, L, max_window):
    nsrc, stride = src.shape
    d_src = torch.from_numpy(src).cuda()
    d_rep = torch.full((len(hdr), stride), 0x77, dtype=torch.uint8, device="cuda")
    d_hdr = torch.from_numpy(hdr.view(np.uint8).copy()).cuda()
    ctx.sw_encode(d_src, d_rep, d_hdr, nsrc=nsrc, nrep=len(hdr), sym_len=L, stride=stride,
                  max_window=max_window)
    torch.cuda.synchronize()
    return d_rep.cpu().numpy()


def schedules(nsrc, rng):
    """name -> (headers, max_window)"""
    out = {}
    out["k8w32"] = (N.sw_schedule(nsrc, 8, 32, key0=65500), 32)
    out["k3w10"] = (N.sw_schedule(nsrc, 3, 10, key0=7, dt=5), 10)
    out["k1w255"] = (N.sw_schedule(nsrc, 1, 255, key0=1), 255)
    out["k4w16_dt0"] = (N.sw_schedule(nsrc, 4, 16, key0=3, dt=0), 16)
    # step longer than the window: gaps no window covers
    out["k40w32"] = ([(max(0, (t + 1) * 40 - 32), min(32, (t + 1) * 40), t, 15)
                      for t in range(nsrc // 40)], 32)
    # windows in random order and sizes
    h = []
    for t in range(300):
        nss = int(rng.integers(1, 49))
        h.append((int(rng.integers(0, nsrc - nss + 1)), nss, t, int(rng.integers(0, 16))))
    out["random"] = (h, 48)
    # the same window over and over (every repair overlaps every other)
    out["repeat"] = ([(100, 30, t, 15) for t in range(150)], 30)
    # a regular stream with some windows moved far away
    base = N.sw_schedule(nsrc, 8, 32, key0=100)
    moved = list(base)
    for t in range(5, len(moved), 9):
        fss, nss, key, dt = moved[t]
        moved[t] = ((fss + 333) % (nsrc - nss), nss, key, dt)
    out["moved"] = (moved, 32)
    out["ragged"] = (base[:-3], 32)
    return out


NSRC = 1200
CASES = list(schedules(NSRC, np.random.default_rng(0)).keys())


@pytest.mark.parametrize("L", [1, 17, 40, 1200, 9000])
@pytest.mark.parametrize("name", CASES)
def test_stream_encode_vs_oracle(ctxs, name, L):
    sched, mw = schedules(NSRC, np.random.default_rng(0))[name]
    if L == 9000 and name in ("k1w255", "random"):
        pytest.skip("covered at smaller symbols (oracle time)")
    stride = O.round_up(L, 16)
    src = stream(NSRC, L, stride, L + len(name))
    hdr = hdr_array(sched)
    o = O.sw_encode(src, hdr, L)
    for mode in MODES:
        g = gpu_encode(ctxs[mode], src, hdr, L, mw)
        assert np.array_equal(g[:, :L], o[:, :L]), f"sw_stream {mode}"


def test_stream_encode_empty_and_clipped(ctxs):
    """Device headers are clipped to [0, nsrc) and max_window; an empty window
    gives a zero repair, between non-empty ones of the same segment."""
    nsrc, L = 300, 64
    src = stream(nsrc, L, 64, 9)
    h = N.sw_schedule(nsrc, 8, 32, key0=4)
    raw = list(h)
    raw[10] = (nsrc + 5, 8, 77, 15)      # starts past the end: empty
    raw[11] = (nsrc - 3, 20, 78, 15)     # clipped to 3 sources
    raw[20] = (h[20][0], 200, 79, 15)    # clipped to max_window
    clipped = list(raw)
    clipped[11] = (nsrc - 3, 3, 78, 15)
    clipped[20] = (h[20][0], 32, 79, 15)
    for mode in MODES[1:]:
        g = gpu_encode(ctxs[mode], src, hdr_array(raw), L, 32)
        keep = [t for t in range(len(raw)) if t != 10]
        o = O.sw_encode(src, hdr_array([clipped[t] for t in keep]), L)
        assert np.array_equal(g[keep, :L], o[:, :L])
        assert not g[10, :L].any()


@pytest.mark.parametrize("nrep", [1, 63, 64, 65, 1000])
def test_stream_encode_segment_edges(ctxs, nrep):
    """Repair counts around the segment size (64) and one repair alone."""
    k, W, L = 8, 32, 100
    nsrc = (nrep + 4) * k
    src = stream(nsrc, L, 112, nrep)
    hdr = hdr_array(N.sw_schedule(nsrc, k, W, key0=nrep)[:nrep])
    o = O.sw_encode(src, hdr, L)
    for mode in MODES[1:]:
        assert np.array_equal(gpu_encode(ctxs[mode], src, hdr, L, W)[:, :L], o[:, :L])


def test_stream_tuning_values():
    c = fecgpu.Context()
    try:
        for v in MODES:
            c.set_tuning("sw_stream", v)
        for v in (-1, 7):
            with pytest.raises(fecgpu.FecError):
                c.set_tuning("sw_stream", v)
    finally:
        c.close()
