"""BASELINE configs[0]: four in-process HotStuff replicas
(dchess/replica.py) replaying the scripted game of tests/golden/oracle_golden.json
through proposal -> quorum -> decision -> commit.  Each replica has its own
dc_ctx and checks every move with dc_validate_batch(n = 1), the signature and
owner with dc_verify_tx_batch(n = 1), commits with dc_apply_batch(n = 1) and
compares game-state hashes from dc_state_hash (checked against the GameState
mirror's host keccak on every commit).

Transactions are signed client-side with the test-only oracle (oracle/txsig.py,
as the frontend does, chess/src/app/play/page.tsx:37-44); player names are the
players' public keys, as the owner check requires (hotstuff.rs:141-148)."""
import json
import os
import sys

import numpy as np
import pytest

import dchess
import oracle_lib as O
from dchess import replica as R

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import txsig as T  # noqa: E402

pytestmark = pytest.mark.gpu

OG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
D_WHITE, D_BLACK = 0x1F00DCAFE, 0x2BADBEEF7
WHITE, BLACK = T.pubkey_hex(D_WHITE), T.pubkey_hex(D_BLACK)


def signed_tx(fx, fy, tx_, ty, turn, tamper=False):
    d = D_WHITE if turn == 0 else D_BLACK
    r, s = T.sign(d, T.message_hash(WHITE, BLACK, (fx, fy, tx_, ty)))
    sig = T.sig_hex(r, s)
    if tamper:
        sig = sig[:-2] + ("00" if sig[-2:] != "00" else "01")
    return {"white_player": WHITE, "black_player": BLACK, "game_state_hash": None,
            "action": [{"x": fx, "y": fy}, {"x": tx_, "y": ty}], "signature": sig,
            "pub_key": WHITE if turn == 0 else BLACK}


@pytest.fixture(scope="module")
def engines():
    es = [dchess.Engine(0) for _ in range(R.PEERS)]
    yield es
    for e in es:
        e.close()


def cluster(engines):
    it = iter(engines)
    bus, reps = R.make_cluster(engine_factory=lambda: next(it))
    for r in reps:
        r.start_game(WHITE, BLACK)
    return bus, reps


def test_four_replicas_commit_the_scripted_game(engines):
    g = OG["replica_game"]
    bus, reps = cluster(engines)
    turn = 0
    accepted = []
    for ply, (fx, fy, tx_, ty) in enumerate(g["moves"]):
        entry = reps[ply % R.PEERS]
        ok = entry.transact(signed_tx(fx, fy, tx_, ty, turn))
        bus.run()
        assert ok == (g["verdicts"][ply] == 0), ply
        if ok:
            turn ^= 1
            accepted.append(ply)
    n_ok = sum(v == 0 for v in g["verdicts"])
    assert len(accepted) == n_ok
    for r in reps:
        assert len(r.committed) == n_ok and r.committed == reps[0].committed
        gs = r.db[f"{WHITE}:{BLACK}"]
        assert gs.history == g["history"] and gs.turn == g["turn"]
        cells = [-1 if c is None else c.color * 8 + "PNBRQK".index(c.kind) for row in gs.board for c in row]
        assert cells == g["final_cells"]
        assert r.game_state_hash(f"{WHITE}:{BLACK}") == reps[0].game_state_hash(f"{WHITE}:{BLACK}")
        assert not [x for x in r.rejections if x[0] != "transact"]
    # the three injected illegal moves were turned away at the entry replica, with the reference's texts
    rej = [x[1] for r in reps for x in r.rejections]
    assert sorted(rej) == sorted(dchess.verdict_message(v) for v in (1, 2, 3))
    assert O.digest(np.array(g["final_cells"], np.int8), g["turn"]) == g["final_digest"]
    # n = 1 validations: entry + leader + 3 voters per committed move
    assert sum(r.validate_calls for r in reps) >= 5 * n_ok


def test_bad_signature_and_wrong_owner_rejected(engines):
    bus, reps = cluster(engines)
    assert not reps[1].transact(signed_tx(1, 4, 3, 4, 0, tamper=True))
    tx = signed_tx(1, 4, 3, 4, 0)
    tx["pub_key"] = BLACK  # signed by white, claimed by black: invalid signature for that key
    assert not reps[2].transact(tx)
    bus.run()
    assert all(not r.committed for r in reps)
    reasons = [x[1] for r in reps for x in r.rejections]
    assert reasons == [dchess.sig_verdict_message(dchess.SIG_INVALID)] * 2


def test_byzantine_leader_block_is_not_committed(engines):
    """A leader that proposes an illegal move (skipping its own is_valid_tx):
    every honest replica's n = 1 validation rejects it, so the leader's vote
    alone stays below the > 2N/3 quorum and nothing commits."""
    bus, reps = cluster(engines)
    leader = next(r for r in reps if r.leader() == r.peer_id)
    tx = dict(signed_tx(0, 0, 2, 2, 0), game_state_hash=leader.game_state_hash(f"{WHITE}:{BLACK}"))  # rook a1-c3
    hist = leader.db[f"{WHITE}:{BLACK}"].history
    block = {"view_n": leader.view_n, "previous_block_hash": leader.latest_block_hash, "tx": tx, "history": hist,
             "hash": R.block_hash(leader.view_n, leader.latest_block_hash, hist, tx), "qc": None}
    bus.publish("quorum", leader.peer_id, block)
    leader.state_votes.setdefault(block["hash"], set()).add(leader.peer_id)
    bus.run()
    assert all(not r.committed for r in reps)
    assert sorted(x[1] for r in reps for x in r.rejections) == [dchess.verdict_message(3)] * 3


def test_stale_state_hash_is_rejected(engines):
    bus, reps = cluster(engines)
    entry = reps[0]
    ok = entry.transact(signed_tx(1, 4, 3, 4, 0))
    bus.run()
    assert ok and all(len(r.committed) == 1 for r in reps)
    # a proposal carrying the pre-move hash for the next move: "inequal game states"
    leader = next(r for r in reps if r.leader() == r.peer_id)
    tx = dict(signed_tx(6, 4, 4, 4, 1), game_state_hash="0x" + "11" * 32)
    hist = leader.db[f"{WHITE}:{BLACK}"].history
    block = {"view_n": leader.view_n, "previous_block_hash": leader.latest_block_hash, "tx": tx, "history": hist,
             "hash": R.block_hash(leader.view_n, leader.latest_block_hash, hist, tx), "qc": None}
    bus.publish("quorum", leader.peer_id, block)
    leader.state_votes.setdefault(block["hash"], set()).add(leader.peer_id)
    bus.run()
    assert all(len(r.committed) == 1 for r in reps)
    assert sorted(x[1] for r in reps for x in r.rejections) == ["inequal game states"] * 3


def test_quorum_threshold_with_silent_replicas(engines):
    """> 2N/3 of 4 is 3 votes: one silent replica still commits, two do not."""
    for silent, commits in ((1, True), (2, False)):
        bus, reps = cluster(engines)
        leader = next(r for r in reps if r.leader() == r.peer_id)
        quiet = [r for r in reps if r is not leader][:silent]
        for q in quiet:
            q.on_message = lambda *a, **k: None
        assert leader.transact(signed_tx(1, 4, 3, 4, 0))
        bus.run()
        assert bool(leader.committed) == commits, silent


def test_rejoining_replica_resyncs_history_and_block_hashes(engines):
    """Resync path: after the scripted game commits, a fresh
    dc_ctx rebuilds the game from the leader's committed blocks with one
    dc_replay_info + dc_history_append and reproduces every block hash
    (types.rs:45-55 over the history before each move), the final history and
    the final game-state hash; a tampered block is caught at its index."""
    g = OG["replica_game"]
    bus, reps = cluster(engines)
    turn = 0
    for ply, (fx, fy, tx_, ty) in enumerate(g["moves"]):
        if reps[ply % R.PEERS].transact(signed_tx(fx, fy, tx_, ty, turn)):
            turn ^= 1
        bus.run()
    blocks = reps[0].blocks
    assert len(blocks) == sum(v == 0 for v in g["verdicts"]) > 0
    fresh = dchess.Engine(0)
    try:
        hist, mv, bad = R.resync_game(fresh, blocks)
        assert bad is None and hist == g["history"]
        k = f"{WHITE}:{BLACK}"
        h = fresh.state_hash(mv.reshape(-1, 1), [(WHITE, BLACK)])[0]
        assert "0x" + bytes(h).hex() == reps[0].game_state_hash(k)
        forged = [dict(b) for b in blocks]
        forged[3] = dict(forged[3], view_n=forged[3]["view_n"] + 1)
        assert R.resync_game(fresh, forged)[2] == 3
    finally:
        fresh.close()
