"""FEC frame wire format: QUIC varint SOURCE_ID and REPAIR
frames through the C ABI (host-only code in libfecgpu.so, runs on CPU).
The fec branch's own frame layout is not mounted: wire parity is unpinned."""
import pytest

import fecgpu


@pytest.mark.parametrize("win", [0, 63, 64, 16383, 16384, (1 << 30) - 1, 1 << 30, (1 << 62) - 1])
@pytest.mark.parametrize("idx", [0, 63, 64, 1000])
def test_source_id_round_trip(win, idx):
    b = fecgpu.frame_source_id(win, idx)
    n, f = fecgpu.frame_parse(b + b"trailing")
    assert n == len(b)
    assert f == {"type": fecgpu.FRAME_SOURCE_ID, "win": win, "idx": idx}


def test_varint_sizes_follow_rfc9000():
    # type 0xfec0 needs a 4-byte varint; window/index 1,2,4,8 bytes at the boundaries
    assert len(fecgpu.frame_source_id(0, 0)) == 4 + 1 + 1
    assert len(fecgpu.frame_source_id(64, 0)) == 4 + 2 + 1
    assert len(fecgpu.frame_source_id(1 << 14, 0)) == 4 + 4 + 1
    assert len(fecgpu.frame_source_id(1 << 30, 0)) == 4 + 8 + 1
    # RFC 9000 A.1 example: 0x25 encodes 37 in one byte; 151288809941952652 in 8 bytes
    b = fecgpu.frame_source_id(151288809941952652, 37)
    assert b[4:12] == bytes.fromhex("c2197c5eff14e88c") and b[12] == 0x25


@pytest.mark.parametrize("sym_len", [0, 1, 1200, 9002, 70000])
def test_repair_round_trip(sym_len):
    sym = bytes((i * 7 + 3) & 0xFF for i in range(sym_len))
    b = fecgpu.frame_repair(123456, 32, 8, 7, sym)
    n, f = fecgpu.frame_parse(b)
    assert n == len(b)
    assert f["type"] == fecgpu.FRAME_REPAIR and f["win"] == 123456
    assert (f["k"], f["r"], f["idx"], f["nsrc"]) == (32, 8, 7, 32)
    assert f["payload"] == sym


@pytest.mark.parametrize("nsrc", [1, 5, 31, 32])
def test_repair_nsrc_round_trip(nsrc):
    """A window closed early carries its real source count (padding
    sources are not on the wire, so the receiver must learn which indices exist)."""
    b = fecgpu.frame_repair(77, 32, 8, 2, b"abc", nsrc=nsrc)
    n, f = fecgpu.frame_parse(b)
    assert n == len(b) and f["nsrc"] == nsrc and f["payload"] == b"abc"
    # layout: type(4) | win(2: 77 >= 64) | k | r | nsrc | idx | len | bytes, all varints
    assert b[4:6] == bytes([0x40, 77]) and b[6:11] == bytes([32, 8, nsrc, 2, 3])


def test_abi1_repair_type_rejected():
    """the nsrc-carrying REPAIR layout has its own type (0xfec4); a
    frame of ABI 1's type 0xfec1 (no nsrc field) is rejected, never misparsed."""
    good = fecgpu.frame_repair(5, 16, 4, 1, b"xyz")
    assert good[:4] == bytes([0x80, 0x00, 0xFE, 0xC4])  # 4-byte varint type
    with pytest.raises(fecgpu.FecError) as e:
        fecgpu.frame_parse(bytes([0x80, 0x00, 0xFE, 0xC1]) + good[4:])
    assert e.value.code == fecgpu.ERR_INVALID_ARG


@pytest.mark.parametrize("nsrc", [0, 33])
def test_repair_nsrc_out_of_range(nsrc):
    with pytest.raises(fecgpu.FecError) as e:
        fecgpu.frame_repair(1, 32, 8, 0, b"x", nsrc=nsrc)
    assert e.value.code == fecgpu.ERR_INVALID_ARG
    # and a parsed frame with nsrc > k is rejected
    good = fecgpu.frame_repair(1, 32, 8, 0, b"x", nsrc=32)
    bad = good[:7] + bytes([33]) + good[8:]
    with pytest.raises(fecgpu.FecError) as e:
        fecgpu.frame_parse(bad)
    assert e.value.code == fecgpu.ERR_INVALID_ARG


@pytest.mark.parametrize("win,sym_len", [(0, 0), (1, 1200), (70000, 9002), ((1 << 62) - 1, 70000)])
def test_repair_header_gather_equals_frame(win, sym_len):
    """Header + symbol bytes from a separate buffer (gather send) == the whole frame."""
    sym = bytes((i * 13 + 1) & 0xFF for i in range(sym_len))
    h = fecgpu.frame_repair_header(win, 16, 4, 3, sym_len)
    assert h + sym == fecgpu.frame_repair(win, 16, 4, 3, sym)
    n, f = fecgpu.frame_parse(h + sym)
    assert n == len(h) + sym_len and f["payload"] == sym


def test_repair_header_errors():
    with pytest.raises(fecgpu.FecError):
        fecgpu.frame_repair_header(1, 16, 4, 4, 10)  # idx >= r
    with pytest.raises(fecgpu.FecError):
        fecgpu.frame_repair_header(1 << 62, 16, 4, 0, 10)
    buf = fecgpu.ctypes.create_string_buffer(4)
    assert fecgpu._lib().fecgpu_frame_write_repair_header(buf, 4, 1, 16, 4, 16, 0, 1200) == -2


def test_parse_errors():
    b = fecgpu.frame_repair(5, 4, 2, 1, b"x" * 100)
    for cut in (0, 1, 3, 5, 9, len(b) - 1):
        with pytest.raises(fecgpu.FecError) as e:
            fecgpu.frame_parse(b[:cut])
        assert e.value.code == fecgpu.ERR_BUFFER_TOO_SHORT
    with pytest.raises(fecgpu.FecError) as e:
        fecgpu.frame_parse(bytes([0x01, 0x00, 0x00]))  # unknown frame type
    assert e.value.code == fecgpu.ERR_INVALID_ARG
    with pytest.raises(fecgpu.FecError) as e:
        fecgpu.frame_repair(5, 4, 2, 2, b"x")  # repair index >= r
    assert e.value.code == fecgpu.ERR_INVALID_ARG


def test_stream_of_frames():
    frames = [fecgpu.frame_source_id(w, i) for w in range(3) for i in range(4)]
    frames += [fecgpu.frame_repair(w, 4, 1, 0, bytes([w]) * 50) for w in range(3)]
    blob = b"".join(frames)
    pos, seen = 0, []
    while pos < len(blob):
        n, f = fecgpu.frame_parse(blob[pos:])
        seen.append(f)
        pos += n
    assert len(seen) == len(frames)
    assert [f["payload"] for f in seen if f["type"] == fecgpu.FRAME_REPAIR] == [bytes([w]) * 50 for w in range(3)]


@pytest.mark.parametrize("esi", [0, 63, 64, 1 << 20, (1 << 62) - 1])
def test_sw_source_round_trip(esi):
    b = fecgpu.frame_sw_source(esi)
    n, f = fecgpu.frame_parse(b + b"payload")
    assert n == len(b)
    assert f["type"] == fecgpu.FRAME_SW_SOURCE and f["esi"] == esi


@pytest.mark.parametrize("hdr", [(0, 1, 0, 15), (123456789, 32, 65535, 7), ((1 << 62) - 1, 255, 1, 0)])
@pytest.mark.parametrize("sym_len", [0, 1, 1202])
def test_sw_repair_round_trip(hdr, sym_len):
    sym = bytes((i * 7) & 0xFF for i in range(sym_len))
    b = fecgpu.frame_sw_repair(hdr, sym)
    n, f = fecgpu.frame_parse(b + b"x")
    assert n == len(b)
    assert f["type"] == fecgpu.FRAME_SW_REPAIR and f["hdr"] == hdr and f["payload"] == sym
    # RFC 8681 repair FEC payload ID fields, QUIC varints: type 0xfec3 is 4 bytes
    assert b[:4] == bytes.fromhex("8000fec3")


def test_sw_repair_errors():
    for bad in [(0, 0, 0, 15), (0, 256, 0, 15), (0, 8, 0, 16), (1 << 62, 8, 0, 15)]:
        with pytest.raises(fecgpu.FecError):
            fecgpu.frame_sw_repair(bad, b"abc")
    b = fecgpu.frame_sw_repair((5, 8, 9, 15), b"0123456789")
    with pytest.raises(fecgpu.FecError):
        fecgpu.frame_parse(b[:-1])   # truncated payload
