"""Host model of gcm_chunk_kernel's chunk claims (nebula_amd/csrc/aes_gcm.hip):
workgroup b owns chunks b, b + G, b + 2G, ... below nstat, its waves draw them from an LDS cursor
(the first 16 without it), and with NEB_CHUNK_STEAL the last nch / 8 chunks are drawn from one
cursor per XCD (blockIdx mod 8), partition x holding chunks nstat + x + 8d. Every chunk must be run
exactly once, whatever order the waves draw in."""
import random

import pytest

WAVES = 16
STEAL = 8  # sched.hpp NEB_CHUNK_STEAL


def run_claims(nch, G, seed):
    rng = random.Random(seed)
    ndyn = nch // STEAL if (G >= 8 and nch >= 32 * G) else 0
    nstat = nch - ndyn
    xcur = [0] * 8
    wg_cur = {}
    done = []

    def chunk_of(b, k):
        return b + k * G

    def claim(b):
        k = chunk_of(b, wg_cur[b])
        wg_cur[b] += 1
        if k >= nstat:
            x = b & 7
            k = nstat + x + 8 * xcur[x]
            xcur[x] += 1
        return k

    waves = []
    for b in range(G):
        if b >= nch:  # the kernel's early return: the workgroup owns no chunk
            continue
        wg_cur[b] = WAVES
        for w in range(WAVES):
            waves.append([b, chunk_of(b, w)])
    # random interleaving: each step one live wave finishes its chunk and claims the next
    live = [wv for wv in waves if wv[1] < nch]
    while live:
        wv = live[rng.randrange(len(live))]
        done.append(wv[1])
        wv[1] = claim(wv[0])
        if wv[1] >= nch:
            live.remove(wv)
    return done, ndyn


@pytest.mark.parametrize("nch,G", [(5888, 256), (8192, 256), (46000, 256), (46001, 256), (300, 8),
                                   (257, 256), (1, 256), (100, 4), (4096, 8), (4097, 9)])
def test_every_chunk_runs_once(nch, G):
    for seed in range(3):
        done, ndyn = run_claims(nch, G, seed)
        assert sorted(done) == list(range(nch))
    if nch >= 32 * G and G >= 8:
        assert ndyn == nch // STEAL


def test_first_chunk_of_every_wave_is_owned():
    # the kernel starts each wave on chunk_of(wave) without a claim: it must lie below nstat
    for G in (8, 64, 256):
        for nch in (32 * G, 32 * G + 7, 100 * G):
            nstat = nch - nch // STEAL
            assert (G - 1) + (WAVES - 1) * G < nstat
