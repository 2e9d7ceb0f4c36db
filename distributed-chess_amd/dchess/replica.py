"""In-process HotStuff replicas around the GPU state-transition check (SURVEY §7
step 9, BASELINE configs[0] "C1").

The reference's consensus (core/src/consensus/hotstuff.rs, core/src/network/
p2p.rs, core/src/network/backend.rs) is out of scope; this module restates
only its control flow, so that the drop-in calls it makes are exercised the
way a replica makes them:

  client --transact--> entry replica           backend.rs:65-108
     is_valid_tx (validate n=1 + signature + owner), game_state_hash,
     publish "proposal"; the leader broadcasts the block itself
  leader: broadcast_block                      p2p.rs:144-177
     is_valid_tx, Block{view_n, previous_block_hash, history, tx, hash},
     publish "quorum", vote for itself
  every other replica: handle_quorum_event     p2p.rs:179-216
     approve_proposal (view, leader, previous hash, block hash,
     is_valid_tx, game_state_hash == its own state hash)
     hotstuff.rs:75-125; vote; publish "decision"
  leader: handle_decision_event / handle_commitment   p2p.rs:218-274
     once votes > 2N/3 (hotstuff.rs:215, p2p.rs:247): QC, publish
     "commit", view_n = block.view_n + 1, commit_block
  replicas: handle_commit_event                p2p.rs:276-291
     commit_block: is_valid_qc (> 2N/3 of its own recorded votes),
     block hash, apply_move (hotstuff.rs:31-73)

Every rule or cryptographic check is one libdchess call with n = 1 on the
replica's own dc_ctx: the move through dc_validate_batch (GameState mirror,
chess.rs:82-98), the signature and owner through dc_verify_tx_batch
(hotstuff.rs:139-148, 168-208), the commit through dc_apply_batch
(chess.rs:43-80), the state hash through dc_state_hash (keccak256 of the
serde_json GameState, hotstuff.rs:153-166) -- cross-checked against the
GameState mirror's host keccak on every commit.  Gossip is a synchronous
in-process bus that, like gossipsub, never delivers a node's message to
itself.  Not restated: the view-change timer (hotstuff.rs:243-262), libp2p,
tonic, and the reference's known faults (the self-deadlock on the apply-reject
path, hotstuff.rs:37/54; panics on missing games and short actions) -- here
a failed apply is reported and the game left unchanged.
"""
import json

import numpy as np

import dchess

PEERS = 4                # core/src/main.rs:29
ZERO_HASH = "0x" + "00" * 32


def _threshold_ok(n_votes, peers=PEERS):
    return n_votes > (2 * peers) // 3  # hotstuff.rs:215, p2p.rs:247


def tx_json(tx):
    """serde_json of the prost Transaction (core/proto/query.proto:37-44: fields in
    declaration order, Option::None as null)."""
    return json.dumps({"white_player": tx["white_player"], "black_player": tx["black_player"],
                       "game_state_hash": tx.get("game_state_hash"),
                       "action": [{"x": a["x"], "y": a["y"]} for a in tx["action"]],
                       "signature": tx["signature"], "pub_key": tx["pub_key"]},
                      separators=(",", ":"), ensure_ascii=False)


def block_hash(view_n, previous_block_hash, history, tx):
    """BlockBuilder::build's hash: keccak256(serde_json(BlockBuilder)) (types.rs:45-55)."""
    body = ('{"view_n":%d,"previous_block_hash":"%s","history":%s,"tx":%s}'
            % (view_n, previous_block_hash, json.dumps(history, ensure_ascii=False), tx_json(tx)))
    return "0x" + dchess.keccak256(body.encode()).hex()


class Bus:
    """Synchronous gossip: publish() delivers to every other replica, in order."""

    def __init__(self):
        self.replicas = []
        self.queue = []
        self.log = []

    def publish(self, topic, source, payload):
        self.log.append((topic, source))
        for r in self.replicas:
            if r.peer_id != source:
                self.queue.append((r, topic, source, payload))

    def run(self):
        while self.queue:
            r, topic, source, payload = self.queue.pop(0)
            r.on_message(topic, source, payload)


class Replica:
    def __init__(self, peer_id, bus, engine=None, check_signatures=True):
        self.peer_id = peer_id
        self.bus = bus
        self.engine = engine or dchess.Engine(0)
        self.check_signatures = check_signatures
        self.db = {}             # game key -> dchess.GameState (mirror on this replica's dc_ctx)
        self.moves = {}          # game key -> committed move words (for dc_state_hash)
        self.view_n = 0
        self.latest_block_hash = ZERO_HASH
        self.state_votes = {}    # block hash -> set of peer ids
        self.committed = []      # block hashes, in commit order
        self.blocks = []         # the committed blocks themselves (a rejoining peer's resync source)
        self.rejections = []     # (where, reason)
        self.validate_calls = 0
        bus.replicas.append(self)

    # ------------------------------------------------------------ helpers
    def leader(self):
        peers = sorted(r.peer_id for r in self.bus.replicas)
        return peers[self.view_n % len(peers)]                  # hotstuff.rs:20-29 (PEERS = cluster size)

    @staticmethod
    def key(tx):
        return f'{tx["white_player"]}:{tx["black_player"]}'

    def start_game(self, white, black):                        # hotstuff.rs:225-234
        k = f"{white}:{black}"
        if k in self.db:
            raise dchess.AppError("already in game")
        self.db[k] = dchess.GameState(white, black, self.engine)
        self.moves[k] = []

    def game_state_hash(self, k):
        """calculate_game_state_hash (hotstuff.rs:153-166) on the GPU: the game
        replayed from GameState::new through its committed moves, then
        keccak256(serde_json(GameState)) (dc_state_hash, n_games = 1)."""
        g = self.db[k]
        mv = np.array(self.moves[k], np.uint16).reshape(-1, 1)
        h = self.engine.state_hash(mv, [(g.white_player, g.black_player)])[0]
        return "0x" + bytes(h).hex()

    # --------------------------------------------------------- the checks
    def is_valid_tx(self, tx):                                 # hotstuff.rs:127-151
        """None if valid, else the reason (AppError text)."""
        k = self.key(tx)
        game = self.db.get(k)
        if game is None:
            return "no such game"
        if len(tx["action"]) < 2:
            return "action needs two positions"                # the reference panics (hotstuff.rs:138)
        a, b = tx["action"][0], tx["action"][1]
        self.validate_calls += 1
        try:
            game.validate_move(dchess.Position(a["x"], a["y"]), dchess.Position(b["x"], b["y"]))  # n = 1
        except dchess.AppError as e:
            return str(e)
        except IndexError:
            return "position out of range"                     # the reference panics (chess.rs:85,92)
        if self.check_signatures:
            blob, off, acts, turns = dchess.pack_txs(
                [(tx["white_player"], tx["black_player"], tx["signature"], tx["pub_key"])],
                np.array([[a["x"], a["y"], b["x"], b["y"]]], np.uint32), np.array([game.turn], np.int8))
            v = int(self.engine.verify_txs(blob, off, acts, turns)[0])  # signature, then owner (n = 1)
            if v != dchess.SIG_OK:
                return dchess.sig_verdict_message(v)
        return None

    # ------------------------------------------------------------ client
    def transact(self, tx):                                    # backend.rs:65-108
        reason = self.is_valid_tx(tx)
        if reason is not None:
            self.rejections.append(("transact", reason))
            return False
        tx = dict(tx, game_state_hash=self.game_state_hash(self.key(tx)))
        self.bus.publish("proposal", self.peer_id, tx)
        if self.leader() == self.peer_id:
            self.broadcast_block(tx)
        return True

    def broadcast_block(self, tx):                             # p2p.rs:144-177
        reason = self.is_valid_tx(tx)
        if reason is not None:
            self.rejections.append(("broadcast", reason))
            return
        hist = self.db[self.key(tx)].history
        block = {"view_n": self.view_n, "previous_block_hash": self.latest_block_hash, "tx": tx, "history": hist,
                 "hash": block_hash(self.view_n, self.latest_block_hash, hist, tx), "qc": None}
        self.bus.publish("quorum", self.peer_id, block)
        self.state_votes.setdefault(block["hash"], set()).add(self.peer_id)

    # ----------------------------------------------------------- handlers
    def on_message(self, topic, source, payload):
        if topic == "proposal":                                # p2p.rs:133-142
            if self.leader() == self.peer_id:
                self.broadcast_block(payload)
        elif topic == "quorum":
            self.on_quorum(payload, source)
        elif topic == "decision":
            self.on_decision(payload, source)
        elif topic == "commit":
            self.on_commit(payload, source)

    def approve_proposal(self, block, source):                 # hotstuff.rs:75-125
        if self.view_n != block["view_n"]:
            return "invalid view"
        if source != self.leader():
            return "incorrect leader"
        if self.latest_block_hash != block["previous_block_hash"]:
            return "invalid block"
        k = self.key(block["tx"])
        if k not in self.db:
            return "no such game"                              # the reference unwraps (hotstuff.rs:101)
        real = block_hash(block["view_n"], block["previous_block_hash"], self.db[k].history, block["tx"])
        if real != block["hash"]:
            return "invalid block"
        reason = self.is_valid_tx(block["tx"])
        if reason is not None:
            return reason
        if block["tx"].get("game_state_hash") != self.game_state_hash(k):
            return "inequal game states"
        return None

    def on_quorum(self, block, source):                        # p2p.rs:179-216
        reason = self.approve_proposal(block, source)
        self.state_votes.setdefault(block["hash"], set()).add(source)
        if reason is None:
            self.state_votes[block["hash"]].add(self.peer_id)
        else:
            self.rejections.append(("approve", reason))
        self.bus.publish("decision", self.peer_id, {"block": block, "decision": reason is None})

    def on_decision(self, commit, source):                     # p2p.rs:218-238
        if commit["decision"]:
            self.state_votes.setdefault(commit["block"]["hash"], set()).add(source)
        if self.leader() == self.peer_id:
            self.handle_commitment(commit)

    def handle_commitment(self, commit):                       # p2p.rs:240-274
        b = commit["block"]
        votes = self.state_votes.get(b["hash"], set())
        if self.view_n == b["view_n"] and _threshold_ok(len(votes), len(self.bus.replicas)):
            b = dict(b, qc={"block_hash": b["hash"], "signature": sorted(votes)})
            self.bus.publish("commit", self.peer_id, b)
            self.view_n = b["view_n"] + 1
            self.commit_block(b)

    def on_commit(self, block, source):                        # p2p.rs:276-291
        if self.view_n == block["view_n"] and self.leader() == source:
            self.view_n = block["view_n"] + 1
            self.commit_block(block)

    def commit_block(self, block):                             # hotstuff.rs:31-73
        qc = block.get("qc")
        if qc is None:
            return self.rejections.append(("commit", "invalid qc"))
        votes = self.state_votes.get(qc["block_hash"], set())  # is_valid_qc, hotstuff.rs:210-223
        if not _threshold_ok(len(votes & set(qc["signature"])), len(self.bus.replicas)):
            return self.rejections.append(("commit", "invalid qc"))
        k = self.key(block["tx"])
        g = self.db.get(k)
        if g is None:
            return self.rejections.append(("commit", "no such game"))
        real = block_hash(block["view_n"], block["previous_block_hash"], g.history, block["tx"])
        if real != block["hash"] or qc["block_hash"] != block["hash"]:
            return self.rejections.append(("commit", "invalid block"))
        a, b = block["tx"]["action"][0], block["tx"]["action"][1]
        try:
            g.apply_move(dchess.Position(a["x"], a["y"]), dchess.Position(b["x"], b["y"]))  # dc_apply_batch, n = 1
        except (dchess.AppError, IndexError) as e:
            return self.rejections.append(("commit", str(e)))  # the game is left unchanged
        self.moves[k].append(dchess.move_pack(a["x"], a["y"], b["x"], b["y"]))
        # the GPU hash of the replayed game must equal the mirror's host keccak
        if self.game_state_hash(k) != g.state_hash():
            raise AssertionError(f"{self.peer_id}: dc_state_hash disagrees with the GameState mirror")
        self.latest_block_hash = block["hash"]
        self.committed.append(block["hash"])
        self.blocks.append(block)


def resync_game(engine, blocks, history=""):
    """A replica that missed a game's commits rebuilds it from the committed
    blocks (in commit order) in one GPU replay instead of commit_block's
    per-block apply_move + update_history (hotstuff.rs:41-56): dc_replay_info
    replays the blocks' moves and reports each ply's moved kind and capture
    flag, dc_history_append turns them into update_history's text
    (chess.rs:127-184), and every block's hash -- BlockBuilder over the
    history BEFORE its move (types.rs:45-55, built in commit_block
    hotstuff.rs:41-46) -- is checked against the rebuilt prefix.
    Returns (final history, the moves as uint16, the first block index whose
    hash or verdict disagrees or None)."""
    mv = np.array([dchess.move_pack(b["tx"]["action"][0]["x"], b["tx"]["action"][0]["y"],
                                    b["tx"]["action"][1]["x"], b["tx"]["action"][1]["y"]) for b in blocks],
                  np.uint16)
    if len(mv) == 0:
        return history, mv, None
    _, _, info, st = engine.replay_info(mv.reshape(-1, 1), want_bitmap=False, want_digests=False)
    info = info[:, 0]
    before = history
    for i, b in enumerate(blocks):
        if info[i] == 0xFF:      # a committed block's move must be legal in the replayed game
            return before, mv, i
        if block_hash(b["view_n"], b["previous_block_hash"], before, b["tx"]) != b["hash"]:
            return before, mv, i
        before = dchess.history_append(before, mv[i:i + 1], info[i:i + 1])
    return before, mv, None


def make_cluster(n=PEERS, check_signatures=True, engine_factory=None):
    """n replicas on one bus, each with its own dc_ctx (one per HotStuff peer)."""
    bus = Bus()
    reps = [Replica(f"peer{i}", bus, (engine_factory or (lambda: dchess.Engine(0)))(), check_signatures)
            for i in range(n)]
    return bus, reps
