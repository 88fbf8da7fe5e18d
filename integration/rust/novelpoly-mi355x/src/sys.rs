//! Raw bindings: one `extern "C"` item per entry point of include/novelpoly.h
//! (what `bindgen include/novelpoly.h` emits, written out so the crate needs no
//! build-time bindgen).  Keep in step with the header; tests/test_abi.py checks
//! the header against the library's exports.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

/// `np_code_params` (novelpoly.h; CodeParams, mod.rs:24-33).
#[repr(C)]
#[derive(Debug, Clone, Copy, Default, PartialEq, Eq)]
pub struct np_code_params {
	pub n: usize,
	pub k: usize,
	pub wanted_n: usize,
}

/// `np_payload_status`: per-payload outcome of a device batch reconstruct.
#[repr(C)]
#[derive(Debug, Clone, Copy, Default, PartialEq, Eq)]
pub struct np_payload_status {
	pub status: i32,
	pub have: u32,
}

/// Opaque `np_ctx` (one per GPU).
#[repr(C)]
pub struct np_ctx {
	_private: [u8; 0],
}

pub const NP_OK: c_int = 0;
pub const NP_ERR_WANTED_SHARD_COUNT_TOO_HIGH: c_int = 1;
pub const NP_ERR_WANTED_SHARD_COUNT_TOO_LOW: c_int = 2;
pub const NP_ERR_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW: c_int = 3;
pub const NP_ERR_PAYLOAD_SIZE_IS_ZERO: c_int = 4;
pub const NP_ERR_NEED_MORE_SHARDS: c_int = 5;
pub const NP_ERR_PARAMETER_MUST_BE_POWER_OF_2: c_int = 6;
pub const NP_ERR_INCONSISTENT_SHARD_LENGTHS: c_int = 7;
pub const NP_ERR_EMPTY_SHARD: c_int = 8;
pub const NP_ERR_INVALID_ARGUMENT: c_int = 100;
pub const NP_ERR_DEVICE: c_int = 101;
pub const NP_ERR_ALLOC: c_int = 102;
pub const NP_ERR_NO_DEVICE: c_int = 103;

extern "C" {
	pub fn np_last_error_detail(out: *mut usize);
	pub fn np_last_error_site() -> *const c_char;
	pub fn np_status_message(status: c_int) -> *const c_char;

	pub fn np_recoverability_subset_size(n_wanted_shards: usize) -> usize;
	pub fn np_derive_parameters(n_wanted: usize, k_wanted: usize, out: *mut np_code_params) -> c_int;
	pub fn np_params_new(n: usize, k: usize, wanted_n: usize, out: *mut np_code_params) -> c_int;
	pub fn np_shard_len(params: *const np_code_params, payload_size: usize) -> usize;
	pub fn np_is_fast_path(params: *const np_code_params) -> c_int;

	pub fn np_ctx_create(device: c_int, out: *mut *mut np_ctx) -> c_int;
	pub fn np_ctx_destroy(ctx: *mut np_ctx);
	pub fn np_ctx_stream(ctx: *mut np_ctx) -> *mut c_void;
	pub fn np_ctx_device(ctx: *mut np_ctx) -> c_int;
	pub fn np_ctx_synchronize(ctx: *mut np_ctx) -> c_int;
	pub fn np_debug_bounds_check(ctx: *mut np_ctx, out: *mut u32) -> c_int;
	pub fn np_pin_registry_stats(out: *mut usize);

	pub fn np_encode(
		ctx: *mut np_ctx,
		payload: *const u8,
		payload_len: usize,
		n_min: usize,
		shards_out: *mut u8,
		shard_len: usize,
	) -> c_int;
	pub fn np_rs_encode(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		payload: *const u8,
		payload_len: usize,
		shards_out: *mut u8,
		shard_len: usize,
	) -> c_int;
	pub fn np_reconstruct(
		ctx: *mut np_ctx,
		shards: *const *const u8,
		shard_lens: *const usize,
		n_received: usize,
		validator_count: usize,
		out: *mut u8,
		out_capacity: usize,
		out_len: *mut usize,
	) -> c_int;
	pub fn np_rs_reconstruct(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		shards: *const *const u8,
		shard_lens: *const usize,
		n_received: usize,
		out: *mut u8,
		out_capacity: usize,
		out_len: *mut usize,
	) -> c_int;
	pub fn np_rs_reconstruct_from_systematic(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		chunks: *const *const u8,
		chunk_lens: *const usize,
		n_chunks: usize,
		out: *mut u8,
		out_capacity: usize,
		out_len: *mut usize,
	) -> c_int;

	pub fn np_encode_batch_dev(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_payloads: *const u8,
		payload_len: usize,
		payload_stride: usize,
		batch: usize,
		d_shards: *mut u8,
		batch_stride: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_reconstruct_batch_dev(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		present: *const u8,
		batch: usize,
		d_out: *mut u8,
		out_stride: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_reconstruct_batch_dev3(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		d_present: *const u8,
		d_locators: *const u16,
		batch: usize,
		d_out: *mut u8,
		out_stride: usize,
		d_status: *mut np_payload_status,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_reconstruct_batch_dev2(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		d_present: *const u8,
		d_locators: *const u16,
		batch: usize,
		d_out: *mut u8,
		out_stride: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_reconstruct_codewords_batch_dev(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		d_present: *const u8,
		batch: usize,
		d_out: *mut u8,
		out_stride: usize,
		d_status: *mut np_payload_status,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_reconstruct_from_systematic_batch_dev(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		d_shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		batch: usize,
		d_out: *mut u8,
		out_stride: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_error_locator_dev(
		ctx: *mut np_ctx,
		n: usize,
		d_present: *const u8,
		batch: usize,
		d_locators: *mut u16,
		stream: *mut c_void,
	) -> c_int;

	pub fn np_encode_batch_host(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		payloads: *const u8,
		payload_len: usize,
		payload_stride: usize,
		batch: usize,
		shards: *mut u8,
		batch_stride: usize,
	) -> c_int;
	pub fn np_reconstruct_batch_host(
		ctx: *mut np_ctx,
		params: *const np_code_params,
		shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		present: *const u8,
		batch: usize,
		out: *mut u8,
		out_stride: usize,
	) -> c_int;

	pub fn np_batch_split(batch: usize, ndev: usize, i: usize, begin: *mut usize, count: *mut usize);
	pub fn np_encode_batch_multi(
		ctxs: *const *mut np_ctx,
		nctx: usize,
		params: *const np_code_params,
		d_payloads: *const *const u8,
		payload_len: usize,
		payload_stride: usize,
		batch: usize,
		d_shards: *const *mut u8,
		batch_stride: usize,
	) -> c_int;
	pub fn np_reconstruct_batch_multi(
		ctxs: *const *mut np_ctx,
		nctx: usize,
		params: *const np_code_params,
		d_shards: *const *const u8,
		shard_len: usize,
		batch_stride: usize,
		d_present: *const *const u8,
		batch: usize,
		d_out: *const *mut u8,
		out_stride: usize,
		d_status: *const *mut np_payload_status,
	) -> c_int;
	pub fn np_encode_batch_host_multi(
		ctxs: *const *mut np_ctx,
		nctx: usize,
		params: *const np_code_params,
		payloads: *const u8,
		payload_len: usize,
		payload_stride: usize,
		batch: usize,
		shards: *mut u8,
		batch_stride: usize,
	) -> c_int;
	pub fn np_reconstruct_batch_host_multi(
		ctxs: *const *mut np_ctx,
		nctx: usize,
		params: *const np_code_params,
		shards: *const u8,
		shard_len: usize,
		batch_stride: usize,
		present: *const u8,
		batch: usize,
		out: *mut u8,
		out_stride: usize,
	) -> c_int;

	pub fn np_afft_dev(ctx: *mut np_ctx, d_data: *mut u16, size: usize, index: usize, cols: usize, stream: *mut c_void) -> c_int;
	pub fn np_inverse_afft_dev(
		ctx: *mut np_ctx,
		d_data: *mut u16,
		size: usize,
		index: usize,
		cols: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_walsh_dev(ctx: *mut np_ctx, d_data: *mut u16, size: usize, stream: *mut c_void) -> c_int;
	pub fn np_mul_dev(
		ctx: *mut np_ctx,
		d_a: *const u16,
		d_m: *const u16,
		d_out: *mut u16,
		count: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_encode_low_dev(
		ctx: *mut np_ctx,
		d_data: *const u16,
		k: usize,
		d_codeword: *mut u16,
		n: usize,
		cols: usize,
		stream: *mut c_void,
	) -> c_int;
	pub fn np_decode_main_dev(
		ctx: *mut np_ctx,
		d_codeword: *mut u16,
		recover_up_to: usize,
		d_present: *const u8,
		d_locator: *const u16,
		n: usize,
		cols: usize,
		stream: *mut c_void,
	) -> c_int;

	pub fn np_version() -> *const c_char;
}
