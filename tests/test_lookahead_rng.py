"""The two-point Woodcock lookahead's RNG restore (csrc/cvr_wpool.hip, "Woodcock
steps ... two points at a time"): after the four draws of a group, the state
after the first point's two draws is (s2, s3, v0, v1, v2) of the current state
with d - 2*362437, where s2, s3 are v0, v1 saved after those two draws.  XORWOW
(cuRAND's, Rng.h:22-30) shifts its five words by one per draw, so this holds
for every state; checked here on random states with a plain restatement of the
transition (the GPU parity tests cover it end to end)."""
import random

M = 0xFFFFFFFF


def xorwow_next(s):
    v0, v1, v2, v3, v4, d = s
    t = (v0 ^ (v0 >> 2)) & M
    n = (v4 ^ ((v4 << 4) & M)) ^ (t ^ ((t << 1) & M))
    return [v1, v2, v3, v4, n & M, (d + 362437) & M]


def restore_two_back(s_now, s2, s3):
    v0, v1, v2, _, _, d = s_now
    return [s2, s3, v0, v1, v2, (d - 2 * 362437) & M]


def test_restore_equals_state_after_first_point():
    rnd = random.Random(1234)
    for _ in range(2000):
        s0 = [rnd.getrandbits(32) for _ in range(6)]
        s1 = xorwow_next(xorwow_next(s0))  # the first point's xi and test value
        s2, s3 = s1[0], s1[1]
        s_end = xorwow_next(xorwow_next(s1))  # the second point's draws
        assert restore_two_back(s_end, s2, s3) == s1


def test_restore_then_redraw_gives_the_dropped_numbers_again():
    # a path that ends at the first point and later continues (e.g. after a null
    # collision decided in the event code) must see the second point's numbers again
    rnd = random.Random(99)
    for _ in range(500):
        s0 = [rnd.getrandbits(32) for _ in range(6)]
        s1 = xorwow_next(xorwow_next(s0))
        s_end = xorwow_next(xorwow_next(s1))
        back = restore_two_back(s_end, s1[0], s1[1])
        assert xorwow_next(xorwow_next(back)) == s_end
