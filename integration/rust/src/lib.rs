//! UNVERIFIED (no cargo in this image).  Raw bindings of include/dchess.h plus
//! a safe `Validator` with the reference's validate/apply call shape
//! (core/src/chess.rs:43-98).  See INTEGRATION.md.
#![allow(non_camel_case_types)]
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
#[derive(Default, Debug)]
pub struct dc_replay_stats {
    pub validated: u64,
    pub accepted: u64,
    pub rejected: u64,
    pub digest_sum: u64,
    pub digest_xor: u64,
}

pub enum dc_ctx {}

pub const DC_RULES_REF: u32 = 0;
pub const DC_RULES_FIDE: u32 = 1;
pub const DC_V_OK: u8 = 0;
pub const DC_V_NO_PIECE: u8 = 1;
pub const DC_V_WRONG_TURN: u8 = 2;
pub const DC_V_ILLEGAL: u8 = 3;
pub const DC_V_OOR: u8 = 4;
pub const DC_CELL_EMPTY: i8 = -1;

extern "C" {
    pub fn dc_ctx_create(device: c_int, out: *mut *mut dc_ctx) -> c_int;
    pub fn dc_ctx_destroy(ctx: *mut dc_ctx) -> c_int;
    pub fn dc_strerror(status: c_int) -> *const c_char;
    pub fn dc_verdict_message(v: u8) -> *const c_char;
    pub fn dc_startpos(out: *mut dc_pos) -> c_int;
    pub fn dc_pos_from_cells(cells: *const i8, turn: u8, out: *mut dc_pos) -> c_int;
    pub fn dc_pos_to_cells(pos: *const dc_pos, cells: *mut i8, turn: *mut u8) -> c_int;
    pub fn dc_move_pack(fx: u32, fy: u32, tx: u32, ty: u32) -> u16;
    pub fn dc_validate_batch(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, moves: *const u16, n: u32,
                             verdicts: *mut u8) -> c_int;
    pub fn dc_apply_batch(ctx: *mut dc_ctx, rules: u32, pos: *mut dc_pos, moves: *const u16, n: u32,
                          verdicts: *mut u8, info: *mut u8) -> c_int;
    pub fn dc_replay(ctx: *mut dc_ctx, rules: u32, start: *const dc_pos, moves: *const u16, n_games: u32,
                     n_plies: u32, bitmap: *mut u64, digests: *mut u64, stats: *mut dc_replay_stats) -> c_int;
    pub fn dc_gen_games(ctx: *mut dc_ctx, rules: u32, seed: u64, first_game: u64, n_games: u32, n_plies: u32,
                        noise_per_256: u32, out: *mut u16) -> c_int;
    pub fn dc_perft(ctx: *mut dc_ctx, rules: u32, pos: *const dc_pos, depth: u32, divide: *mut u64,
                    root_moves: *mut u16, n_root: *mut u32, total: *mut u64) -> c_int;
    pub fn dc_device_alloc(ctx: *mut dc_ctx, bytes: usize, d_ptr: *mut *mut c_void) -> c_int;
    pub fn dc_device_free(ctx: *mut dc_ctx, d_ptr: *mut c_void) -> c_int;
    pub fn dc_keccak256(data: *const c_void, len: usize, out: *mut u8) -> c_int;
    pub fn dc_state_hash(ctx: *mut dc_ctx, start: *const dc_pos, history: *const c_char, names: *const c_char,
                         names_off: *const u32, moves: *const u16, n_games: u32, n_plies: u32,
                         hashes: *mut u8) -> c_int;
    pub fn dc_verify_tx_batch(ctx: *mut dc_ctx, strings: *const c_char, str_off: *const u32, actions: *const u32,
                              turns: *const i8, n: u32, verdicts: *mut u8) -> c_int;
    pub fn dc_sig_verdict_message(v: u8) -> *const c_char;
    pub fn dc_replay_shard_range(n_games: u64, shard: u32, n_shards: u32, first: *mut u64, count: *mut u64) -> c_int;
    pub fn dc_multi_replay(devices: *const c_int, n_devices: c_int, rules: u32, seed: u64, n_games: u64,
                           n_plies: u32, noise_per_256: u32, bitmap: *mut u64, stats: *mut dc_replay_stats) -> c_int;
}

/// One device context (one gfx950 GPU, one HIP stream).  Not Sync: keep one per thread.
pub struct Validator(*mut dc_ctx);

impl Validator {
    pub fn new(device: i32) -> Result<Self, String> {
        let mut c = std::ptr::null_mut();
        let s = unsafe { dc_ctx_create(device, &mut c) };
        if s != 0 {
            return Err(unsafe { std::ffi::CStr::from_ptr(dc_strerror(s)) }.to_string_lossy().into());
        }
        Ok(Validator(c))
    }

    /// Verdict of one (from, to) pair, as GameState::validate_move (chess.rs:82-98):
    /// Ok(()) or the reference's reject string.
    pub fn validate(&self, pos: &dc_pos, from: (u32, u32), to: (u32, u32)) -> Result<(), String> {
        let mv = unsafe { dc_move_pack(from.0, from.1, to.0, to.1) };
        let mut v = 0u8;
        let s = unsafe { dc_validate_batch(self.0, DC_RULES_REF, pos, &mv, 1, &mut v) };
        assert_eq!(s, 0, "dc_validate_batch failed");
        match v {
            DC_V_OK => Ok(()),
            _ => Err(unsafe { std::ffi::CStr::from_ptr(dc_verdict_message(v)) }.to_string_lossy().into()),
        }
    }
}

impl Drop for Validator {
    fn drop(&mut self) {
        unsafe { dc_ctx_destroy(self.0) };
    }
}
