"""K3's per-row staging ring (vp8l_transforms.hip pred_wavefront): a row's 24-column ring holds its
un-emitted outputs and its staged inputs.  Inputs arrive as aligned 32-byte blocks (8 columns),
one per chunk per row -- block c - r/4 for row r, the block holding the chunk's last column --
and outputs leave as aligned 16-column blocks once complete.  This replays that schedule for
every row of a band over several widths and checks the invariant the kernel relies on: every
column a chunk reads is still the staged input, and every column an emission reads is that
column's output (nothing overwritten early).  CPU only; no device code involved."""
import pytest

K_BAND, K_CHUNK, K_OUT_COLS = 64, 8, 24


def replay_row(r, width):
    ring = [None] * K_OUT_COLS
    steps = width + 2 * (K_BAND - 1)
    nch = 2 * ((steps + 2 * K_CHUNK - 1) // (2 * K_CHUNK))
    emitted = 0
    for c in range(nch):
        a = c - (r >> 2)  # the aligned block staged before chunk c
        for k in range(K_CHUNK):
            ring[(K_CHUNK * a + k) % K_OUT_COLS] = ("in", K_CHUNK * a + k)
        s = K_CHUNK * c - 2 * r  # the chunk's first column for row r
        for x in range(s, s + K_CHUNK):
            if 0 <= x < width:
                assert ring[x % K_OUT_COLS] == ("in", x), (r, c, x, ring[x % K_OUT_COLS])
                ring[x % K_OUT_COLS] = ("out", x)
        while 16 * emitted + 16 <= s + K_CHUNK:  # blocks completed by this chunk
            for x in range(16 * emitted, 16 * emitted + 16):
                if x < width:
                    assert ring[x % K_OUT_COLS] == ("out", x), (r, c, x, ring[x % K_OUT_COLS])
            emitted += 1


@pytest.mark.parametrize("width", [1, 7, 16, 33, 250, 2048])
def test_k3_ring_schedule(width):
    for r in range(K_BAND):
        replay_row(r, width)
