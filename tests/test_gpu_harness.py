"""The reference's own experiment on the GPU engine (SEQ schedule).

`send_messages` / `one_message_test` (src/gossiper.rs:173-323) drive the
literal harness order, which the engine runs as GS_SCHED_SEQ.  Every
iteration's metrics (nodes/msgs missed, the five summed Statistics, rounds,
first round of full spread) must equal the CPU oracle's on the same Philox
schedule (integer work: exact), and their averages must reproduce the
reference's only published numbers (README.md:5 -> img/evaluate_result.png,
1000 iterations), within the tolerance the oracle itself meets
(tests/test_oracle_network.py).
"""
import numpy as np
import pytest

from oracle_lib import SCHED_SEQ, OracleNet
from test_oracle_network import README

pytestmark = pytest.mark.gpu

SEED = 0xC0FFEE


@pytest.mark.parametrize("n,iters", [(20, 300), (200, 150), (2000, 30)])
def test_one_message_seq_matches_oracle_and_readme(engine, n, iters):
    net = engine.Network(n, 1, seed=SEED, schedule="SEQ")
    orc = OracleNet(n, 1, seed=SEED)
    acc = np.zeros(4)
    try:
        for it in range(iters):
            nm, mm, st, rounds_run, round_full = engine.send_messages(net, 1)
            m = orc.send_messages(1, SCHED_SEQ)
            got = (nm, mm, st.rounds, st.empty_pull_sent, st.empty_push_sent,
                   st.full_message_sent, st.full_message_received, rounds_run, round_full)
            exp = (m.nodes_missed, m.msgs_missed, m.stats.rounds, m.stats.empty_pull_sent,
                   m.stats.empty_push_sent, m.stats.full_message_sent,
                   m.stats.full_message_received, m.rounds_run, m.round_full)
            assert got == exp, f"iteration {it}: gpu {got} oracle {exp}"
            acc += [st.rounds, st.empty_pull_sent + st.empty_push_sent, st.full_message_sent, mm]
    finally:
        net.close()
        orc.close()
    rounds, empties, full, _ = acc / iters
    e_rounds, e_empty, e_full = README[n]
    tol = 0.03 if iters >= 100 else 0.05
    assert int(rounds) == e_rounds or abs(rounds - e_rounds) < 0.75
    assert abs(empties - e_empty) / e_empty < tol
    assert abs(full - e_full) / e_full < tol


@pytest.mark.parametrize("n,R,num,schedule", [(200, 16, 10, "SEQ"), (300, 70, 64, "2P"),
                                               (150, 8, 3, "SEQ")])
def test_send_messages_fewer_rumors_than_slots(engine, n, R, num, schedule):
    # send_messages(gossipers, num_of_msgs) with more rumor slots than rumors:
    # "complete" means messages().len() == num_of_msgs (src/gossiper.rs:246),
    # so round_full must follow the oracle's (or_send_messages) exactly
    from oracle_lib import SCHED_2P
    net = engine.Network(n, R, seed=SEED, schedule=schedule)
    orc = OracleNet(n, R, seed=SEED)
    try:
        fulls = 0
        for it in range(4):
            nm, mm, st, rounds_run, round_full = engine.send_messages(net, num)
            m = orc.send_messages(num, SCHED_SEQ if schedule == "SEQ" else SCHED_2P)
            got = (nm, mm, st.rounds, st.empty_pull_sent, st.empty_push_sent,
                   st.full_message_sent, st.full_message_received, rounds_run, round_full)
            exp = (m.nodes_missed, m.msgs_missed, m.stats.rounds, m.stats.empty_pull_sent,
                   m.stats.empty_push_sent, m.stats.full_message_sent,
                   m.stats.full_message_received, m.rounds_run, m.round_full)
            assert got == exp, f"iteration {it}: gpu {got} oracle {exp}"
            fulls += round_full > 0
        assert fulls >= 1
    finally:
        net.close()
        orc.close()


def _oracle_one_message_lines(n, iters, msgs, schedule):
    """The AVERAGE / MIN / MAX lines one_message_test prints
    (src/gossiper.rs:270-343), computed from the oracle's send_messages."""
    from oracle_lib import SCHED_2P
    orc = OracleNet(n, msgs, seed=0x5AFE6055)
    mets = [orc.send_messages(msgs, SCHED_SEQ if schedule == "SEQ" else SCHED_2P)
            for _ in range(iters)]
    orc.close()
    fields = ("rounds", "empty_pull_sent", "empty_push_sent", "full_message_sent",
              "full_message_received")
    stats = [[getattr(m.stats, f) for f in fields] for m in mets]
    avg = [sum(c) // iters for c in zip(*stats)]           # u64 integer division
    mn = [min(c) for c in zip(*stats)]
    mx = [max(c) for c in zip(*stats)]
    nm = [m.nodes_missed for m in mets]
    mm = [m.msgs_missed for m in mets]

    def line(nmv, mmv, s):
        return ("rounds: %d, empty_pulls: %d, empty_pushes: %d, full_msgs_sent: %d, "
                "msgs_missed: %g (%.2f%%), nodes_missed: %g (%.2f%%)"
                % (s[0], s[1], s[2], s[3], mmv, 100.0 * mmv / n / msgs, nmv,
                   100.0 * nmv / n / msgs))
    return ["AVERAGE ---- " + line(sum(nm) / iters, sum(mm) / iters, avg),
            "MIN -------- " + line(float(min(nm)), float(min(mm)), mn),
            "MAX -------- " + line(float(max(nm)), float(max(mm)), mx)]


@pytest.mark.parametrize("n,iters,msgs,schedule", [(20, 200, 1, "SEQ"), (200, 40, 1, "SEQ"),
                                                    (200, 10, 5, "2P")])
def test_one_message_example_binary(engine, n, iters, msgs, schedule):
    # the compiled C++ driver examples/one_message_test (one_message_test and
    # print_metric, src/gossiper.rs:261-344, through include/safe_gossip.hpp)
    # prints exactly the AVERAGE / MIN / MAX lines the oracle's iterations give
    import subprocess
    from safe_gossip_amd.build import REPO_DIR, build_examples
    exe = [e for e in build_examples() if e.endswith("one_message_test")][0]
    out = subprocess.run([exe, str(n), str(iters), str(msgs), schedule], capture_output=True,
                         text=True, timeout=300, cwd=REPO_DIR)
    assert out.returncode == 0, out.stderr
    got = [ln.strip() for ln in out.stdout.splitlines() if "----" in ln]
    assert got == _oracle_one_message_lines(n, iters, msgs, schedule)
