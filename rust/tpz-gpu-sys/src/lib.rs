//! `extern "C"` binding of `libtpz_gpu.so`, the C ABI declared in `include/tpz_gpu.h`.
//!
//! Every item mirrors one declaration of the header (same name, same field order, same
//! argument types); `tests/test_rust_binding.py` parses both files and fails when they drift
//! apart. The safe layer topazdb uses sits in `rust/topazdb-gpu` (`Block::from_columns`,
//! `SsTable::read_blocks_gpu`), which replaces the reference's `SsTable::read_block` +
//! `Block::decode` (`src/table.rs:154-164`, `src/block.rs:46-65`) for batches of blocks.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

/// `tpz_err`: an API failure (a per-block outcome is a `TPZ_BLOCK_*` status, not an error).
pub type TpzErr = c_int;
pub const TPZ_SUCCESS: TpzErr = 0;
pub const TPZ_ERR_INVALID_ARG: TpzErr = -1;
pub const TPZ_ERR_HIP: TpzErr = -2;
pub const TPZ_ERR_NO_DEVICE: TpzErr = -3;
pub const TPZ_ERR_NOMEM: TpzErr = -4;
pub const TPZ_ERR_INTERNAL: TpzErr = -5;
pub const TPZ_ERR_SIZES: TpzErr = -6;

/// `tpz_block_status`, one byte per block in `d_status` / `h_status`.
pub const TPZ_BLOCK_OK: u8 = 0;
pub const TPZ_BLOCK_EMPTY: u8 = 1;
pub const TPZ_BLOCK_BAD_TAG: u8 = 2;
pub const TPZ_BLOCK_UNSUPPORTED_CODEC: u8 = 3;
pub const TPZ_BLOCK_CHECKSUM_MISMATCH: u8 = 4;
pub const TPZ_BLOCK_MALFORMED: u8 = 5;
pub const TPZ_BLOCK_OK_SPILLED: u8 = 6;
pub const TPZ_BLOCK_SPILL_FULL: u8 = 7;
pub const TPZ_BLOCK_CODEC_ERROR: u8 = 8;
pub const TPZ_BLOCK_BAD_ENTRY: u8 = 9;

/// `tpz_entry_class`: per-entry class byte of a `TPZ_BLOCK_BAD_ENTRY` block's spill record.
pub const TPZ_ENTRY_OK: u8 = 0;
pub const TPZ_ENTRY_BAD_VALUE: u8 = 1;
pub const TPZ_ENTRY_BAD_KEY: u8 = 2;

pub const TPZ_ABI_VERSION: c_int = 6;
pub const TPZ_LDS_BLOCK_BYTES: u32 = 94192;
pub const TPZ_BIGWAVE_BLOCK_BYTES: u32 = 0x40000000;
pub const TPZ_PLAN_ASYNC_MAX_BLOCK: u32 = 10242;

/// `tpz_batch`: blocks (or ranges, or files) back to back in HBM; block i is
/// `d_src[d_ext[i] .. d_ext[i + 1])`.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzBatch {
    pub d_src: *const u8,
    pub d_ext: *const u64,
    pub n_blocks: u32,
    pub src_bytes: u64,
}

/// `tpz_columns`: the decode's outputs in HBM (slotted layout: block i's keys, then its values
/// from the next 16-byte boundary, at `tpz_layout_slot_base(ext[i], i)`).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzColumns {
    pub d_data: *mut u8,
    pub d_ends: *mut u32,
    pub d_count: *mut u32,
    pub d_status: *mut u8,
    pub d_crc: *mut u32,
    pub d_spill: *mut u8,
    pub spill_cap: u64,
    pub d_spill_off: *mut u64,
    pub d_spill_used: *mut u64,
    pub d_entry_first: *const u64,
}

/// `tpz_flat_columns`: the flat layout (one dense key column and one dense value column for the
/// batch, exact `{kend, vend}` pairs); `d_first` from `tpz_flat_layout`.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzFlatColumns {
    pub d_keys: *mut u8,
    pub d_values: *mut u8,
    pub d_ends: *mut u32,
    pub d_first: *const u64,
    pub d_count: *mut u32,
    pub d_status: *mut u8,
    pub d_crc: *mut u32,
    pub d_spill: *mut u8,
    pub spill_cap: u64,
    pub d_spill_off: *mut u64,
    pub d_spill_used: *mut u64,
}

/// `tpz_host_columns`: `tpz_decode_blocks_host`'s outputs in host memory.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzHostColumns {
    pub h_data: *mut u8,
    pub h_ends: *mut u32,
    pub ends_cap: u64,
    pub h_first: *mut u64,
    pub h_count: *mut u32,
    pub h_status: *mut u8,
    pub h_crc: *mut u32,
    pub h_spill: *mut u8,
    pub spill_cap: u64,
    pub h_spill_off: *mut u64,
    pub h_spill_used: *mut u64,
    pub h_dext: *mut u64,
    pub data_cap: u64,
}

/// `tpz_table`: a table decoded on the device plus its block metas' first keys.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzTable {
    pub d_first_keys: *const u8,
    pub d_first_pos: *const u64,
    pub d_ext: *const u64,
    pub n_blocks: u32,
    pub d_data: *const u8,
    pub d_ends: *const u32,
    pub d_count: *const u32,
    pub d_status: *const u8,
    pub d_spill: *const u8,
    pub d_spill_off: *const u64,
    pub d_entry_first: *const u64,
}

/// `tpz_entries`: sorted entries in HBM (the write side).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct TpzEntries {
    pub d_keys: *const u8,
    pub d_kpos: *const u64,
    pub d_vals: *const u8,
    pub d_vpos: *const u64,
    pub n_entries: u32,
    pub key_bytes: u64,
    pub val_bytes: u64,
}

/// `tpz_ctx` (opaque).
#[repr(C)]
pub struct TpzCtx {
    _private: [u8; 0],
}

extern "C" {
    pub fn tpz_abi_version() -> c_int;
    pub fn tpz_layout_slot_base(ext_i: u64, i: u64) -> u64;
    pub fn tpz_layout_value_start(key_bytes: u64) -> u64;
    pub fn tpz_layout_entry_base(ext_i: u64, i: u64) -> u64;
    pub fn tpz_layout_data_capacity(src_bytes: u64, n_blocks: u64) -> u64;
    pub fn tpz_layout_entry_capacity(src_bytes: u64, n_blocks: u64) -> u64;
    pub fn tpz_layout_spill_stream(n: u64) -> u64;
    pub fn tpz_layout_spill_classes(n: u64, k: u64, v: u64) -> u64;
    pub fn tpz_ctx_create(device: c_int, out: *mut *mut TpzCtx) -> TpzErr;
    pub fn tpz_ctx_destroy(ctx: *mut TpzCtx);
    pub fn tpz_ctx_reserve(ctx: *mut TpzCtx, max_blocks: u32, stream: *mut c_void) -> TpzErr;
    pub fn tpz_decode_blocks(ctx: *mut TpzCtx, batch: *const TpzBatch, out: *const TpzColumns,
                             stream: *mut c_void) -> TpzErr;
    pub fn tpz_decode_check(ctx: *mut TpzCtx, stream: *mut c_void) -> TpzErr;
    pub fn tpz_entry_first(ctx: *mut TpzCtx, batch: *const TpzBatch, d_first: *mut u64,
                           stream: *mut c_void) -> TpzErr;
    pub fn tpz_pack_ends(ctx: *mut TpzCtx, batch: *const TpzBatch, cols: *const TpzColumns,
                         d_first: *const u64, d_dense: *mut u32, stream: *mut c_void) -> TpzErr;
    pub fn tpz_layout_compress_bound(src_bytes: u64, n_blocks: u64) -> u64;
    pub fn tpz_compress_blocks(ctx: *mut TpzCtx, batch: *const TpzBatch, codec: u32, d_dst: *mut u8,
                               d_dst_ext: *mut u64, stream: *mut c_void) -> TpzErr;
    pub fn tpz_flat_layout(ctx: *mut TpzCtx, batch: *const TpzBatch, d_first: *mut u64,
                           stream: *mut c_void) -> TpzErr;
    pub fn tpz_decode_blocks_flat(ctx: *mut TpzCtx, batch: *const TpzBatch,
                                  out: *const TpzFlatColumns, stream: *mut c_void) -> TpzErr;
    pub fn tpz_host_decoded_bound(h_src: *const u8, h_ext: *const u64, n_blocks: u32,
                                  bound: *mut u64) -> TpzErr;
    pub fn tpz_decode_blocks_host(ctx: *mut TpzCtx, h_src: *const u8, h_ext: *const u64,
                                  n_blocks: u32, out: *const TpzHostColumns,
                                  chunk_blocks: u32) -> TpzErr;
    pub fn tpz_verify_blocks_host(ctx: *mut TpzCtx, h_src: *const u8, h_ext: *const u64,
                                  n_blocks: u32, h_status: *mut u8, h_crc: *mut u32,
                                  h_count: *mut u32, h_plain: *mut u8, plain_cap: u64,
                                  h_dext: *mut u64, chunk_blocks: u32) -> TpzErr;
    pub fn tpz_crc32_ranges(ctx: *mut TpzCtx, ranges: *const TpzBatch, d_crc: *mut u32,
                            stream: *mut c_void) -> TpzErr;
    pub fn tpz_verify_files(ctx: *mut TpzCtx, files: *const TpzBatch, d_crc: *mut u32,
                            d_status: *mut u8, stream: *mut c_void) -> TpzErr;
    pub fn tpz_verify_files_flat_layout(ctx: *mut TpzCtx, blocks: *const TpzBatch,
                                        d_file_block: *const u32, tails: *const TpzBatch,
                                        d_crc: *mut u32, d_status: *mut u8, d_first: *mut u64,
                                        stream: *mut c_void) -> TpzErr;
    pub fn tpz_decompressed_sizes(ctx: *mut TpzCtx, batch: *const TpzBatch, d_size: *mut u64,
                                  stream: *mut c_void) -> TpzErr;
    pub fn tpz_decompressed_sizes_claimed(ctx: *mut TpzCtx, batch: *const TpzBatch,
                                          d_size: *mut u64, stream: *mut c_void) -> TpzErr;
    pub fn tpz_decompress_check(ctx: *mut TpzCtx, stream: *mut c_void) -> TpzErr;
    pub fn tpz_decompress_blocks(ctx: *mut TpzCtx, batch: *const TpzBatch, d_dst: *mut u8,
                                 d_dst_ext: *const u64, d_status: *mut u8,
                                 stream: *mut c_void) -> TpzErr;
    pub fn tpz_seek_keys(ctx: *mut TpzCtx, table: *const TpzTable, d_keys: *const u8,
                         d_key_pos: *const u64, n_keys: u32, d_block: *mut u32,
                         d_entry: *mut u32, d_status: *mut u8, d_valid: *mut u8,
                         stream: *mut c_void) -> TpzErr;
    pub fn tpz_bloom_may_contain(ctx: *mut TpzCtx, d_filter: *const u8, filter_len: u64,
                                 d_keys: *const u8, d_key_pos: *const u64, n_keys: u32,
                                 d_out: *mut u8, stream: *mut c_void) -> TpzErr;
    pub fn tpz_host_xxh3_64(h_buf: *const u8, len: u64) -> u64;
    pub fn tpz_bloom_geometry(n_keys: u64, fpp: f64, filter_len: *mut u64, k: *mut u32) -> TpzErr;
    pub fn tpz_bloom_build(ctx: *mut TpzCtx, d_keys: *const u8, d_key_pos: *const u64,
                           n_keys: u32, fpp: f64, d_filter: *mut u8, stream: *mut c_void) -> TpzErr;
    pub fn tpz_plan_blocks(ctx: *mut TpzCtx, entries: *const TpzEntries, block_size: u32,
                           d_first: *mut u32, d_ext: *mut u64, h_n_blocks: *mut u32,
                           h_bad_entry: *mut u64, stream: *mut c_void) -> TpzErr;
    pub fn tpz_encode_blocks(ctx: *mut TpzCtx, entries: *const TpzEntries, d_first: *const u32,
                             d_ext: *const u64, n_blocks: u32, d_out: *mut u8,
                             stream: *mut c_void) -> TpzErr;
    pub fn tpz_plan_blocks_async(ctx: *mut TpzCtx, entries: *const TpzEntries, block_size: u32,
                                 d_first: *mut u32, d_ext: *mut u64, d_info: *mut u32,
                                 stream: *mut c_void) -> TpzErr;
    pub fn tpz_encode_blocks_async(ctx: *mut TpzCtx, entries: *const TpzEntries,
                                   d_first: *const u32, d_ext: *const u64, d_info: *const u32,
                                   d_out: *mut u8, stream: *mut c_void) -> TpzErr;
    pub fn tpz_build_blocks(h_keys: *const u8, h_kpos: *const u64, h_vals: *const u8,
                            h_vpos: *const u64, n_entries: u64, block_size: u32, h_out: *mut u8,
                            out_cap: u64, h_ext: *mut u64, ext_cap: u64, n_blocks: *mut u64,
                            out_len: *mut u64) -> c_int;
    pub fn tpz_snappy_encode_blocks(h_src: *const u8, h_ext: *const u64, n_blocks: u64,
                                    h_out: *mut u8, out_cap: u64, h_out_ext: *mut u64,
                                    out_len: *mut u64) -> c_int;
    pub fn tpz_lz4_encode_blocks(h_src: *const u8, h_ext: *const u64, n_blocks: u64,
                                 h_out: *mut u8, out_cap: u64, h_out_ext: *mut u64,
                                 out_len: *mut u64) -> c_int;
    pub fn tpz_host_crc32(h_buf: *const u8, len: u64) -> u32;
    pub fn tpz_format_block_error(status: c_int, crc_expected: u32, crc_actual: u32,
                                  buf: *mut c_char, cap: usize) -> c_int;
    pub fn tpz_last_error() -> *const c_char;
}

/// The header's inline layout helpers, restated (the exported `tpz_layout_*` functions compute
/// the same values; `tests/test_abi.py` checks those against the header's definitions).
pub mod layout {
    /// Block i's output slot: its keys, then its values from `value_start(K)`.
    pub fn slot_base(ext_i: u64, i: u64) -> u64 {
        ((ext_i + 127) & !127) + 256 * i
    }
    pub fn value_start(key_bytes: u64) -> u64 {
        (key_bytes + 15) & !15
    }
    /// Block i's first {kend, vend} pair in the slotted ends.
    pub fn entry_base(ext_i: u64, i: u64) -> u64 {
        16 * (ext_i / 96 + i)
    }
}
