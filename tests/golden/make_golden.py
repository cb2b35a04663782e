"""Writes the hand-derived known-answer vectors used to pin the CPU oracle.

The reference crate holds no golden vectors (its tests only print,
src/gossiper.rs:299-322), and it cannot be built here (Rust absent), so every
expected value below is derived BY HAND from the cited reference lines; the
derivation is the comment next to each case.  Nothing here is computed by the
oracle or the engine.  Run: python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
A, B, C, D = 0, 1, 2, 3
P14 = (3, 3, 14)  # counter_max, max_c_rounds, max_rounds (e.g. n = 1e6)

# Each case: state (tag, round, our_counter, rounds_in_state_b) -> receive the
# records in order (first one creates when state is A) -> next_round(P).
MESSAGE_STATE = [
    # message_state.rs:51-57 new() = B{0,1}; :99 round 1; :108-112 P empty;
    # :130 0 > 0 false; :136 1 < 3 -> B{1,1}.
    dict(name="new_then_next_round_empty_P", state=[B, 0, 1, 0], records=[], pir=[],
         params=P14, expect=[B, 1, 1, 0]),
    # peer_counters {a:1,b:1}, P={a,b,c}: c gets 0 (:108-112); a,b: 1>=1 and
    # 1<3 -> ge=2; c: 0<1 -> less=1; 2>1 -> our_counter 2 (:130-132).
    dict(name="median_bump", state=[B, 0, 1, 0], records=[[1, 1], [2, 1]], pir=[1, 2, 3],
         params=P14, expect=[B, 1, 2, 0]),
    # any counter >= counter_max -> C{rounds_in_state_b: round, round: 0} (:121-125).
    dict(name="c_copy_moves_to_c", state=[B, 0, 1, 0], records=[[1, 255]], pir=[1],
         params=P14, expect=[C, 0, 0, 1]),
    # round 13 + 1 = 14 >= max_rounds 14 -> D (:99-103).
    dict(name="b_max_rounds_to_d", state=[B, 13, 1, 0], records=[], pir=[], params=P14,
         expect=[D, 0, 0, 0]),
    # our_counter 2, {a:1,b:2}: a less, b ge -> 1 > 1 false -> stays 2 (tie).
    dict(name="median_tie_no_bump", state=[B, 0, 2, 0], records=[[1, 1], [2, 2]], pir=[1, 2],
         params=P14, expect=[B, 1, 2, 0]),
    # C{rib 5, round 0}: round 1 (+5 < 14, 1 < 3) -> C{5,1} (:152-167).
    dict(name="c_round_1", state=[C, 0, 0, 5], records=[], pir=[], params=P14,
         expect=[C, 1, 0, 5]),
    dict(name="c_round_2", state=[C, 1, 0, 5], records=[], pir=[], params=P14,
         expect=[C, 2, 0, 5]),
    # round 3 >= max_c_rounds 3 -> D (:159-161).
    dict(name="c_max_c_rounds_to_d", state=[C, 2, 0, 5], records=[], pir=[], params=P14,
         expect=[D, 0, 0, 0]),
    # C{rib 12}: 1 + 12 = 13 < 14 -> C{12,1}; then 2 + 12 = 14 -> D (:154-156).
    dict(name="c_total_rounds_1", state=[C, 0, 0, 12], records=[], pir=[], params=P14,
         expect=[C, 1, 0, 12]),
    dict(name="c_total_rounds_to_d", state=[C, 1, 0, 12], records=[], pir=[], params=P14,
         expect=[D, 0, 0, 0]),
    # new_from_peer (:62-74): 2 < 3 -> B{0,1}; 3 and 255 -> C{0,0}.  No next_round.
    dict(name="new_from_peer_b", state=[A, 0, 0, 0], records=[[1, 2]], pir=[], params=P14,
         expect=[B, 0, 1, 0], next_round=False),
    dict(name="new_from_peer_c_at_cmax", state=[A, 0, 0, 0], records=[[1, 3]], pir=[],
         params=P14, expect=[C, 0, 0, 0], next_round=False),
    dict(name="new_from_peer_c_255", state=[A, 0, 0, 0], records=[[1, 255]], pir=[],
         params=P14, expect=[C, 0, 0, 0], next_round=False),
    # counter_max 1 (n <= 15): new() -> round 1 < 3, no votes, our_counter 1 >= 1 -> C{1,0}.
    dict(name="cmax1_new_to_c", state=[B, 0, 1, 0], records=[], pir=[], params=[1, 1, 3],
         expect=[C, 0, 0, 1]),
    # received copy at cmax 1 -> C{0,0}; next_round: 1+0 < 3 but 1 >= max_c_rounds 1 -> D.
    dict(name="cmax1_copy_to_d", state=[A, 0, 0, 0], records=[[4, 255]], pir=[4],
         params=[1, 1, 3], expect=[D, 0, 0, 0]),
    # {a:2,b:1,c:1} + zeros for d,e: ge = 3, less = 2 -> bump to 2.
    dict(name="median_five_peers", state=[B, 0, 1, 0], records=[[1, 2], [2, 1], [3, 1]],
         pir=[1, 2, 3, 4, 5], params=P14, expect=[B, 1, 2, 0]),
    # {a:1}, P={a,b}: ge 1, less 1 -> no bump.
    dict(name="median_half", state=[B, 0, 1, 0], records=[[1, 1]], pir=[1, 2], params=P14,
         expect=[B, 1, 1, 0]),
    # B{5,2} {a:2,b:2,c:1}: ge 2 > less 1 -> 3 >= counter_max -> C{rib 6, round 0} (:136-141).
    dict(name="bump_to_cmax_to_c", state=[B, 5, 2, 0], records=[[1, 2], [2, 2], [3, 1]],
         pir=[1, 2, 3], params=P14, expect=[C, 0, 0, 6]),
    # {a:1, b:255}: key order a then b; b >= counter_max -> C{1,0}.
    dict(name="c_copy_after_b_copy", state=[B, 0, 1, 0], records=[[1, 1], [2, 255]],
         pir=[1, 2], params=P14, expect=[C, 0, 0, 1]),
    # D is sticky (:169).
    dict(name="d_sticky", state=[D, 0, 0, 0], records=[[1, 1]], pir=[1], params=P14,
         expect=[D, 0, 0, 0]),
    # receive on C is ignored (:78), then C{2,1} -> C{2,2}.
    dict(name="c_ignores_copies", state=[C, 1, 0, 2], records=[[1, 1]], pir=[1], params=P14,
         expect=[C, 2, 0, 2]),
    # same peer twice: BTreeMap::insert overwrites (:79).  B{0,2}: a=1 then a=2
    # -> a:2 >= 2 -> ge 1 > less 0 -> 3 >= 3 -> C{1,0}.  (No overwrite would
    # leave a:1 < 2 -> B{1,2}.)
    dict(name="same_peer_overwrites", state=[B, 0, 2, 0], records=[[1, 1], [1, 2]], pir=[1],
         params=P14, expect=[C, 0, 0, 1]),
    # max_rounds 1 (n = 2): new() -> round 1 >= 1 -> D.
    dict(name="n2_new_to_d", state=[B, 0, 1, 0], records=[], pir=[], params=[1, 1, 1],
         expect=[D, 0, 0, 0]),
    # three zero votes: less 3 -> B{4,1}.
    dict(name="zero_votes", state=[B, 3, 1, 0], records=[], pir=[1, 2, 3], params=P14,
         expect=[B, 4, 1, 0]),
    # From A: the first copy creates B{0,1} and is NOT recorded (gossip.rs:159-161);
    # its sender is still in P so it votes 0: a:0 less, b:1 ge -> tie -> B{1,1}.
    dict(name="creator_votes_zero", state=[A, 0, 0, 0], records=[[1, 1], [2, 1]], pir=[1, 2],
         params=P14, expect=[B, 1, 1, 0]),
    # From A with a C copy first: C{0,0}; the later B copy is ignored -> C{0,1}.
    dict(name="created_c_ignores", state=[A, 0, 0, 0], records=[[1, 255], [2, 1]], pir=[1, 2],
         params=P14, expect=[C, 1, 0, 0]),
]

OUR_COUNTER = [  # message_state.rs:175-181
    dict(state=[B, 3, 2, 0], expect=2),
    dict(state=[B, 0, 1, 0], expect=1),
    dict(state=[C, 1, 0, 4], expect=255),
    dict(state=[D, 0, 0, 0], expect=-1),
]

PARAMS = [  # gossip.rs:59-64 (f64 ln, ceil, `as u8`, max 1), network_size = n
    dict(n=2, expect=[1, 1, 1]),        # ln ln 2 = -0.37 -> ceil -0 -> 0 -> 1; ln 2 -> 1
    dict(n=3, expect=[1, 1, 2]),        # ln 3 = 1.10 -> 2; ln ln 3 = 0.094 -> 1
    dict(n=8, expect=[1, 1, 3]),        # examples/network.rs size: ln 8 = 2.08 -> 3
    dict(n=15, expect=[1, 1, 3]),       # ln ln 15 = 0.996 -> 1
    dict(n=16, expect=[2, 2, 3]),       # ln ln 16 = 1.0197 -> 2
    dict(n=20, expect=[2, 2, 3]),       # README: ln 20 = 3.00 -> 3, ln ln = 1.10 -> 2
    dict(n=200, expect=[2, 2, 6]),      # ln 5.30 -> 6, ln ln 1.67 -> 2
    dict(n=1618, expect=[2, 2, 8]),     # ln ln 1618 = 1.99998 -> 2
    dict(n=1619, expect=[3, 3, 8]),     # ln ln 1619 = 2.00006 -> 3
    dict(n=2000, expect=[3, 3, 8]),     # README: ln 7.60 -> 8, ln ln 2.03 -> 3
    dict(n=5000, expect=[3, 3, 9]),
    dict(n=10000, expect=[3, 3, 10]),
    dict(n=1000000, expect=[3, 3, 14]),  # config 2/3
    dict(n=16777216, expect=[3, 3, 17]),  # config 4 (2^24)
    dict(n=100000000, expect=[3, 3, 19]),  # config 5
]

# Random123 known-answer vectors for philox4x32-10 (kat_vectors).
PHILOX = [
    dict(ctr=[0, 0, 0, 0], key=[0, 0],
         expect=[0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    dict(ctr=[0xFFFFFFFF] * 4, key=[0xFFFFFFFF] * 2,
         expect=[0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    dict(ctr=[0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], key=[0xA4093822, 0x299F31D0],
         expect=[0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]

# Whole-network known answers (2P schedule; with n = 2 the schedule is forced:
# each node's only peer is the other).
NETWORK = [
    # n=2, params (1,1,1).  Round 1 phase 0: node 0 gets send_new -> B{0,1} ->
    # next_round: round 1 >= max_rounds 1 -> D (message_state.rs:99-103); no
    # live entry -> empty push, empty_push_sent+1 (gossip.rs:105-111); node 1
    # likewise.  Phase 1: each receives an empty push from the other, is_new ->
    # no live entries -> one empty pull, empty_pull_sent+1 (gossip.rs:141-147);
    # empty RPCs are not absorbed (gossip.rs:153).  Node 0 knows the rumor (D),
    # node 1 does not; nothing live was pushed.
    dict(name="n2_dies_at_origin", n=2, R=1, injections={"1": [[0, 0]]}, rounds=1,
         expect_any_live=[False],
         expect_state=[[D << 14], [0]],
         expect_stats=[[1, 1, 1, 0, 0], [1, 1, 1, 0, 0]]),
]


def main():
    data = dict(message_state=MESSAGE_STATE, our_counter=OUR_COUNTER, params=PARAMS,
                philox=PHILOX, network=[c for c in NETWORK])
    with open(os.path.join(HERE, "kat_reference.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("wrote", os.path.join(HERE, "kat_reference.json"))


if __name__ == "__main__":
    main()
