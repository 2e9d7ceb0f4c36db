//! UNVERIFIED (no cargo/rustc in this image; text-checked against
//! include/dchess.h by tests/test_abi.py::test_rust_binding_matches_header).
//!
//! `sys`: every entry point of include/dchess.h, one to one.
//! `Engine`: a safe, panic-free layer -- every non-zero status becomes
//! `DcError`, which the reference maps into its `AppError` (core/src/errors.rs).
//! `apply_move` / `validate_move`: the reference's GameState methods
//! (core/src/chess.rs:43-125) over the proto board flattened to 64 cells.
//! See INTEGRATION.md.
#![allow(non_camel_case_types)]

use std::ffi::{CStr, CString};
use std::os::raw::{c_char, c_int, c_void};

pub mod sys {
    use std::os::raw::{c_char, c_int, c_void};

    #[repr(C)]
    #[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
    pub struct dc_pos {
        pub bb: [u64; 4],
        pub stm: u8,
        pub castle: u8,
        pub ep: i8,
        pub reserved0: u8,
        pub reserved1: u32,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
    pub struct dc_replay_stats {
        pub validated: u64,
        pub accepted: u64,
        pub rejected: u64,
        pub digest_sum: u64,
        pub digest_xor: u64,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Default, Debug)]
    pub struct dc_kernel_stats {
        pub launches: u64,
        pub total_ms: f64,
        pub units: u64,
    }

    pub enum dc_ctx {}

    pub const DC_SUCCESS: c_int = 0;
    pub const DC_EINVAL: c_int = -1;
    pub const DC_EHIP: c_int = -2;
    pub const DC_ENOMEM: c_int = -3;
    pub const DC_ENODEV: c_int = -4;
    pub const DC_ERCCL: c_int = -5;
    pub const DC_EUNSUPPORTED: c_int = -6;
    pub const DC_RULES_REF: u32 = 0;
    pub const DC_RULES_FIDE: u32 = 1;
    pub const DC_V_OK: u8 = 0;
    pub const DC_V_NO_PIECE: u8 = 1;
    pub const DC_V_WRONG_TURN: u8 = 2;
    pub const DC_V_ILLEGAL: u8 = 3;
    pub const DC_V_OOR: u8 = 4;
    pub const DC_MOVE_OOR: u16 = 0x8000;
    pub const DC_MOVE_NONE: u16 = 0xFFFF;
    pub const DC_CELL_EMPTY: i8 = -1;
    pub const DC_SIG_OK: u8 = 0;
    pub const DC_SIG_BAD_SIG_HEX: u8 = 1;
    pub const DC_SIG_BAD_SIG: u8 = 2;
    pub const DC_SIG_BAD_PK_HEX: u8 = 3;
    pub const DC_SIG_BAD_PK: u8 = 4;
    pub const DC_SIG_INVALID: u8 = 5;
    pub const DC_SIG_WRONG_OWNER: u8 = 6;

    extern "C" {
        // context
        pub fn dc_ctx_create(device: c_int, out: *mut *mut dc_ctx) -> c_int;
        pub fn dc_ctx_destroy(ctx: *mut dc_ctx) -> c_int;
        pub fn dc_ctx_device(ctx: *const dc_ctx) -> c_int;
        pub fn dc_ctx_stream(ctx: *mut dc_ctx) -> *mut c_void;
        pub fn dc_strerror(status: c_int) -> *const c_char;
        pub fn dc_verdict_message(verdict: u8) -> *const c_char;
        pub fn dc_version() -> c_int;
        pub fn dc_ctx_set_profiling(ctx: *mut dc_ctx, enable: c_int) -> c_int;
        pub fn dc_ctx_kernel_stats(ctx: *mut dc_ctx, kernel: *const c_char, out: *mut dc_kernel_stats) -> c_int;
        pub fn dc_ctx_reset_stats(ctx: *mut dc_ctx) -> c_int;
        pub fn dc_device_alloc(ctx: *mut dc_ctx, bytes: usize, d_ptr: *mut *mut c_void) -> c_int;
        pub fn dc_device_free(ctx: *mut dc_ctx, d_ptr: *mut c_void) -> c_int;
        pub fn dc_memcpy_h2d(ctx: *mut dc_ctx, d_dst: *mut c_void, src: *const c_void, bytes: usize) -> c_int;
        pub fn dc_memcpy_d2h(ctx: *mut dc_ctx, dst: *mut c_void, d_src: *const c_void, bytes: usize) -> c_int;
        // adapters
        pub fn dc_startpos(out: *mut dc_pos) -> c_int;
        pub fn dc_pos_from_cells(cells: *const i8, turn: u8, out: *mut dc_pos) -> c_int;
        pub fn dc_pos_to_cells(pos: *const dc_pos, cells: *mut i8, turn: *mut u8) -> c_int;
        pub fn dc_pos_from_fen(fen: *const c_char, out: *mut dc_pos) -> c_int;
        pub fn dc_move_pack(from_x: u32, from_y: u32, to_x: u32, to_y: u32) -> u16;
        pub fn dc_move_pack_batch(actions: *const u32, n: u32, moves: *mut u16) -> c_int;
        // validation
        pub fn dc_validate_batch(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, moves: *const u16, n: u32,
                                 verdicts: *mut u8) -> c_int;
        pub fn dc_apply_batch(ctx: *mut dc_ctx, rules: u32, pos: *mut dc_pos, moves: *const u16, n: u32,
                              verdicts: *mut u8, info: *mut u8) -> c_int;
        pub fn dc_live_validator(ctx: *mut dc_ctx, lease_us: u32) -> c_int;
        // replay
        pub fn dc_replay(ctx: *mut dc_ctx, rules: u32, start: *const dc_pos, moves: *const u16, n_games: u32,
                         n_plies: u32, bitmap: *mut u64, digests: *mut u64, stats: *mut dc_replay_stats) -> c_int;
        pub fn dc_replay_device(ctx: *mut dc_ctx, rules: u32, start: *const dc_pos, d_moves: *const u16,
                                n_games: u32, n_plies: u32, d_bitmap: *mut u64, d_digests: *mut u64,
                                stats: *mut dc_replay_stats) -> c_int;
        pub fn dc_replay_info(ctx: *mut dc_ctx, rules: u32, start: *const dc_pos, moves: *const u16, n_games: u32,
                              n_plies: u32, bitmap: *mut u64, digests: *mut u64, info: *mut u8,
                              stats: *mut dc_replay_stats) -> c_int;
        pub fn dc_replay_info_device(ctx: *mut dc_ctx, rules: u32, start: *const dc_pos, d_moves: *const u16,
                                     n_games: u32, n_plies: u32, d_bitmap: *mut u64, d_digests: *mut u64,
                                     d_info: *mut u8, stats: *mut dc_replay_stats) -> c_int;
        pub fn dc_history_append(history: *const c_char, moves: *const u16, info: *const u8, n_plies: u32,
                                 stride: usize, out: *mut c_char, out_cap: usize, out_len: *mut usize) -> c_int;
        pub fn dc_gen_games(ctx: *mut dc_ctx, rules: u32, seed: u64, first_game: u64, n_games: u32, n_plies: u32,
                            noise_per_256: u32, out: *mut u16) -> c_int;
        pub fn dc_gen_games_device(ctx: *mut dc_ctx, rules: u32, seed: u64, first_game: u64, n_games: u32,
                                   n_plies: u32, noise_per_256: u32, d_out: *mut u16) -> c_int;
        // state hash
        pub fn dc_keccak256(data: *const c_void, len: usize, out: *mut u8) -> c_int;
        pub fn dc_state_hash(ctx: *mut dc_ctx, start: *const dc_pos, history: *const c_char, names: *const c_char,
                             names_off: *const u32, moves: *const u16, n_games: u32, n_plies: u32,
                             hashes: *mut u8) -> c_int;
        pub fn dc_state_hash_device(ctx: *mut dc_ctx, start: *const dc_pos, history: *const c_char,
                                    d_names: *const c_char, d_names_off: *const u32, d_moves: *const u16,
                                    n_games: u32, n_plies: u32, d_hashes: *mut u8) -> c_int;
        // transaction signatures
        pub fn dc_verify_tx_batch(ctx: *mut dc_ctx, strings: *const c_char, str_off: *const u32,
                                  actions: *const u32, turns: *const i8, n: u32, verdicts: *mut u8) -> c_int;
        pub fn dc_verify_tx_batch_device(ctx: *mut dc_ctx, d_strings: *const c_char, d_str_off: *const u32,
                                         d_actions: *const u32, d_turns: *const i8, n: u32,
                                         d_verdicts: *mut u8) -> c_int;
        pub fn dc_sig_verdict_message(verdict: u8) -> *const c_char;
        // perft
        pub fn dc_perft(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, depth: u32, divide: *mut u64,
                        root_moves: *mut u16, n_root: *mut u32, total: *mut u64) -> c_int;
        pub fn dc_perft_shard(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, depth: u32, split_depth: u32,
                              shard: u32, n_shards: u32, divide: *mut u64, root_moves: *mut u16,
                              n_root: *mut u32, total: *mut u64) -> c_int;
        pub fn dc_perft_repeat_device(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, depth: u32,
                                      split_depth: u32, shard: u32, n_shards: u32, n_runs: u32,
                                      d_out: *mut u64) -> c_int;
        pub fn dc_perft_batch(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, n_pos: u32, depth: u32,
                              totals: *mut u64, divide: *mut u64, root_moves: *mut u16, root_pos: *mut u8,
                              n_root: *mut u32) -> c_int;
        pub fn dc_perft_batch_repeat_device(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, n_pos: u32,
                                            depth: u32, split_depth: u32, n_runs: u32, d_out: *mut u64) -> c_int;
        pub fn dc_ctx_synchronize(ctx: *mut dc_ctx) -> c_int;
        // multi-GPU
        pub fn dc_multi_perft(devices: *const c_int, n_devices: c_int, rules: u32, pos: *const dc_pos, depth: u32,
                              divide: *mut u64, root_moves: *mut u16, n_root: *mut u32, total: *mut u64) -> c_int;
        pub fn dc_replay_shard_range(n_games: u64, shard: u32, n_shards: u32, first: *mut u64,
                                     count: *mut u64) -> c_int;
        pub fn dc_replay_scatter_shards(n_games: u64, n_shards: u32, n_plies: u32, gathered: *const u64,
                                        bitmap: *mut u64) -> c_int;
        pub fn dc_multi_replay(devices: *const c_int, n_devices: c_int, rules: u32, seed: u64, n_games: u64,
                               n_plies: u32, noise_per_256: u32, bitmap: *mut u64,
                               stats: *mut dc_replay_stats) -> c_int;
    }
}

/// A failed ABI call: the DC_E* status and its dc_strerror text.  Never a
/// rejected move -- that is a verdict (`Verdict`), not an error.
#[derive(Clone, Debug, PartialEq, Eq)]
pub struct DcError {
    pub status: c_int,
    pub what: &'static str,
    pub text: String,
}

impl std::fmt::Display for DcError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "{}: {} ({})", self.what, self.text, self.status)
    }
}
impl std::error::Error for DcError {}

fn cstr(p: *const c_char) -> String {
    if p.is_null() {
        return String::new();
    }
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

fn check(status: c_int, what: &'static str) -> Result<(), DcError> {
    if status == sys::DC_SUCCESS {
        Ok(())
    } else {
        Err(DcError { status, what, text: cstr(unsafe { sys::dc_strerror(status) }) })
    }
}

/// The reference's rejection (core/src/chess.rs:82-125): Ok or the exact text
/// validate_move returns; OOR is the coordinate the reference would panic on.
#[derive(Clone, Debug, PartialEq, Eq)]
pub enum Verdict {
    Ok,
    Rejected(String),
    OutOfRange,
}

fn verdict(v: u8) -> Verdict {
    match v {
        sys::DC_V_OK => Verdict::Ok,
        sys::DC_V_OOR => Verdict::OutOfRange,
        _ => Verdict::Rejected(cstr(unsafe { sys::dc_verdict_message(v) })),
    }
}

/// One device context (one gfx950 GPU, one HIP stream).  Send but not Sync:
/// keep one per thread (e.g. a thread_local per tokio blocking worker).
pub struct Engine(*mut sys::dc_ctx);
unsafe impl Send for Engine {}

impl Engine {
    pub fn new(device: i32) -> Result<Self, DcError> {
        let mut c = std::ptr::null_mut();
        check(unsafe { sys::dc_ctx_create(device, &mut c) }, "dc_ctx_create")?;
        Ok(Engine(c))
    }

    pub fn raw(&self) -> *mut sys::dc_ctx {
        self.0
    }

    /// Opt-in resident validator for this context (dc_live_validator): calls of
    /// at most 64 moves skip the kernel launch while the lease lasts; 0 stops it.
    pub fn live_validator(&self, lease_us: u32) -> Result<(), DcError> {
        check(unsafe { sys::dc_live_validator(self.0, lease_us) }, "dc_live_validator")
    }

    /// validate_move (chess.rs:82) for one (from, to) pair: n = 1, the live consensus call.
    pub fn validate(&self, pos: &sys::dc_pos, from: (u32, u32), to: (u32, u32)) -> Result<Verdict, DcError> {
        let mv = unsafe { sys::dc_move_pack(from.0, from.1, to.0, to.1) };
        let mut v = 0u8;
        check(unsafe { sys::dc_validate_batch(self.0, sys::DC_RULES_REF, pos, &mv, 1, &mut v) },
              "dc_validate_batch")?;
        Ok(verdict(v))
    }

    /// A block's worth of checks at once (is_valid_tx over many transactions).
    pub fn validate_batch(&self, pos: &[sys::dc_pos], moves: &[u16]) -> Result<Vec<Verdict>, DcError> {
        if pos.len() != moves.len() || pos.len() > u32::MAX as usize {
            return Err(DcError { status: sys::DC_EINVAL, what: "validate_batch", text: "length mismatch".into() });
        }
        let mut v = vec![0u8; pos.len()];
        check(unsafe { sys::dc_validate_batch(self.0, sys::DC_RULES_REF, pos.as_ptr(), moves.as_ptr(),
                                              pos.len() as u32, v.as_mut_ptr()) }, "dc_validate_batch")?;
        Ok(v.into_iter().map(verdict).collect())
    }

    /// apply_move (chess.rs:43-80) on the cells of a proto board: validates,
    /// makes the move on the GPU, updates `turn` and appends the history entry
    /// (update_history, chess.rs:127-184, via dc_history_append).  A rejected
    /// move leaves everything untouched and returns its verdict.  Cells of kind
    /// OTHER (6) never move (chess.rs:210), so the caller's kind strings for
    /// them stay valid.
    pub fn apply_move(&self, cells: &mut [i8; 64], turn: &mut u8, history: &mut String, from: (u32, u32),
                      to: (u32, u32)) -> Result<Verdict, DcError> {
        let mut pos = sys::dc_pos::default();
        check(unsafe { sys::dc_pos_from_cells(cells.as_ptr(), *turn, &mut pos) }, "dc_pos_from_cells")?;
        let mv = unsafe { sys::dc_move_pack(from.0, from.1, to.0, to.1) };
        let (mut v, mut info) = (0u8, 0u8);
        check(unsafe { sys::dc_apply_batch(self.0, sys::DC_RULES_REF, &mut pos, &mv, 1, &mut v, &mut info) },
              "dc_apply_batch")?;
        if v != sys::DC_V_OK {
            return Ok(verdict(v));
        }
        let h = history_append(history, &[mv], &[info])?;
        check(unsafe { sys::dc_pos_to_cells(&pos, cells.as_mut_ptr(), turn) }, "dc_pos_to_cells")?;
        *history = h;
        Ok(Verdict::Ok)
    }

    /// Resync: replay a game's committed moves in one call; returns the per-ply
    /// info bytes (0xFF = rejected) and the counters.
    pub fn replay_info(&self, moves: &[u16]) -> Result<(Vec<u8>, sys::dc_replay_stats), DcError> {
        // n_plies is a u32 at the ABI: a longer log is an error, never truncated
        let n_plies = u32::try_from(moves.len()).map_err(|_| DcError {
            status: sys::DC_EINVAL, what: "dc_replay_info", text: "move log longer than u32::MAX plies".into() })?;
        let mut info = vec![0u8; moves.len()];
        let mut st = sys::dc_replay_stats::default();
        check(unsafe { sys::dc_replay_info(self.0, sys::DC_RULES_REF, std::ptr::null(), moves.as_ptr(), 1,
                                           n_plies, std::ptr::null_mut(), std::ptr::null_mut(),
                                           info.as_mut_ptr(), &mut st) }, "dc_replay_info")?;
        Ok((info, st))
    }
}

impl Drop for Engine {
    fn drop(&mut self) {
        let _ = unsafe { sys::dc_ctx_destroy(self.0) };
    }
}

/// update_history over plies (dc_history_append, host only): no panic on any input.
pub fn history_append(history: &str, moves: &[u16], info: &[u8]) -> Result<String, DcError> {
    if moves.len() != info.len() {
        return Err(DcError { status: sys::DC_EINVAL, what: "history_append", text: "length mismatch".into() });
    }
    let h = CString::new(history)
        .map_err(|_| DcError { status: sys::DC_EINVAL, what: "history_append", text: "NUL in history".into() })?;
    let mut len = 0usize;
    check(unsafe { sys::dc_history_append(h.as_ptr(), moves.as_ptr(), info.as_ptr(), moves.len() as u32, 1,
                                          std::ptr::null_mut(), 0, &mut len) }, "dc_history_append")?;
    let mut out = vec![0u8; len + 1];
    check(unsafe { sys::dc_history_append(h.as_ptr(), moves.as_ptr(), info.as_ptr(), moves.len() as u32, 1,
                                          out.as_mut_ptr() as *mut c_char, out.len(), &mut len) },
          "dc_history_append")?;
    out.truncate(len);
    String::from_utf8(out)
        .map_err(|_| DcError { status: sys::DC_EINVAL, what: "history_append", text: "not UTF-8".into() })
}

/// keccak256 (alloy) of one byte string, on the host.
pub fn keccak256(data: &[u8]) -> Result<[u8; 32], DcError> {
    let mut out = [0u8; 32];
    check(unsafe { sys::dc_keccak256(data.as_ptr() as *const c_void, data.len(), out.as_mut_ptr()) },
          "dc_keccak256")?;
    Ok(out)
}
