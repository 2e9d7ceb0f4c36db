"""Host-side pieces of dchess/replica.py (no GPU): the > 2N/3 threshold, the
block hash (keccak256 of serde_json(BlockBuilder), core/src/consensus/types.rs:45-55,
via libdchess's host dc_keccak256) and the gossip bus semantics."""
from dchess import replica as R


def tx(**kw):
    t = {"white_player": "w", "black_player": "b", "game_state_hash": None,
         "action": [{"x": 1, "y": 4}, {"x": 3, "y": 4}], "signature": "s", "pub_key": "w"}
    t.update(kw)
    return t


def test_threshold_is_more_than_two_thirds():
    assert [R._threshold_ok(n) for n in range(5)] == [False, False, False, True, True]  # PEERS = 4
    assert R._threshold_ok(5, peers=7) and not R._threshold_ok(4, peers=7)


def test_tx_json_field_order_and_null():
    assert R.tx_json(tx()) == ('{"white_player":"w","black_player":"b","game_state_hash":null,'
                               '"action":[{"x":1,"y":4},{"x":3,"y":4}],"signature":"s","pub_key":"w"}')


def test_block_hash_binds_every_field():
    h = R.block_hash(0, R.ZERO_HASH, "", tx())
    assert h.startswith("0x") and len(h) == 66 and h == R.block_hash(0, R.ZERO_HASH, "", tx())
    assert h != R.block_hash(1, R.ZERO_HASH, "", tx())
    assert h != R.block_hash(0, "0x" + "11" * 32, "", tx())
    assert h != R.block_hash(0, R.ZERO_HASH, "1. e4", tx())
    assert h != R.block_hash(0, R.ZERO_HASH, "", tx(signature="t"))


def test_bus_never_delivers_to_the_sender():
    bus = R.Bus()

    class Sink:
        def __init__(self, pid):
            self.peer_id, self.got = pid, []

        def on_message(self, topic, source, payload):
            self.got.append((topic, source))

    a, b, c = Sink("a"), Sink("b"), Sink("c")
    bus.replicas = [a, b, c]
    bus.publish("quorum", "a", {})
    bus.run()
    assert a.got == [] and b.got == [("quorum", "a")] and c.got == [("quorum", "a")]
