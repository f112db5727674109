"""The local cluster's side of the multiplexed port-forward tunnel (devspace_amd/localkube/spdy.py):
the same SPDY/3 dictionary as the client (src/kube/spdy.cc, checked by the C++ test
spdy_dictionary_is_the_protocols) and frames that parse wherever the tunnel's WebSocket messages
cut them. The two ends talk to each other in tests/test_e2e_services.py."""
import random
import struct
import zlib

from devspace_amd.localkube import spdy


def test_dictionary_is_the_protocols():
    assert len(spdy.DICTIONARY) == 1423
    assert zlib.adler32(spdy.DICTIONARY) == 0xE3C6A7C2


def test_header_blocks_round_trip_through_one_zlib_stream():
    c = zlib.compressobj(zdict=spdy.DICTIONARY)
    d = zlib.decompressobj(zdict=spdy.DICTIONARY)
    for i in range(5):
        h = {"streamtype": "data" if i % 2 else "error", "port": "8080", "requestid": str(i)}
        block = c.compress(spdy.encode_headers(h)) + c.flush(zlib.Z_SYNC_FLUSH)
        assert spdy.decode_headers(d.decompress(block)) == h


def test_frames_parse_wherever_they_are_cut():
    wire = (spdy.control_frame(spdy.SYN_STREAM, 0, struct.pack(">II", 1, 0) + b"\0\0hdr") +
            spdy.data_frame(1, spdy.FLAG_FIN, bytes(range(256)) * 300) +
            spdy.control_frame(spdy.PING, 0, struct.pack(">I", 9)))
    rng = random.Random(3)
    buf, got, off = bytearray(), [], 0
    while off < len(wire):
        n = rng.randint(1, 5000)
        buf += wire[off:off + n]
        off += n
        got += list(spdy.parse_frames(buf))
    assert [(c, t, f) for c, t, f, _ in got] == [(True, spdy.SYN_STREAM, 0), (False, 1, spdy.FLAG_FIN),
                                                   (True, spdy.PING, 0)]
    assert got[1][3] == bytes(range(256)) * 300 and not buf
