//! MI355X backend for `reed-solomon-novelpoly` (v2.0.0).
//!
//! The functions and types below have the signatures of the crate's own
//! (`novel_poly_basis::{encode, reconstruct}` at encode.rs:6 / reconstruct.rs:4,
//! `CodeParams` / `ReedSolomon` at mod.rs:24-285) and return its `Error`
//! (errors.rs:4-28), so a caller switches by changing the import:
//!
//! ```ignore
//! use novelpoly_mi355x as rs;          // was: use reed_solomon_novelpoly as rs;
//! let shards: Vec<WrappedShard> = rs::encode(&payload, 1024)?;
//! let payload = rs::reconstruct(received, 1024)?;
//! ```
//!
//! The work runs on the GPU through libnovelpoly_hip.so (include/novelpoly.h);
//! results are bit-identical to the crate (the repository's tests/).  The
//! crate's alternative-implementation slot (`src/cxx.rs:23-31`, feature
//! `with-alt-cxx-impl`, both functions `unimplemented!()`) can forward to
//! `encode` / `reconstruct` here unchanged.
//!
//! Batch entry points (`encode_batch`, `reconstruct_batch`, `*_multi`) expose
//! the library's batched host API: many payloads of one shape per call,
//! pipelined over several streams (and over several GPUs for `*_multi`).
//!
//! Not compiled in the repository's CI image (it has no Rust toolchain);
//! tests/test_abi.py checks that `sys.rs` declares every entry point of the
//! header with the same parameter count.

pub mod sys;

use reed_solomon_novelpoly::{Error, Result, Shard};
use std::os::raw::c_int;
use std::sync::{Mutex, OnceLock};

/// One library context (GPU) per device, created on first use.
pub struct Context {
	raw: *mut sys::np_ctx,
}

// The library serialises calls on one context with its own lock.
unsafe impl Send for Context {}
unsafe impl Sync for Context {}

impl Context {
	/// Context on HIP device `device` (-1: the current device).
	pub fn new(device: i32) -> Result<Context> {
		let mut raw = std::ptr::null_mut();
		check(unsafe { sys::np_ctx_create(device as c_int, &mut raw) })?;
		Ok(Context { raw })
	}

	pub fn device(&self) -> i32 {
		unsafe { sys::np_ctx_device(self.raw) }
	}

	pub fn as_raw(&self) -> *mut sys::np_ctx {
		self.raw
	}
}

impl Drop for Context {
	fn drop(&mut self) {
		unsafe { sys::np_ctx_destroy(self.raw) }
	}
}

/// The process-wide default context (device 0), as the free functions use.
/// Panics when no gfx950 device is usable: a build that links this backend
/// has no CPU path to fall back to.
pub fn default_context() -> &'static Context {
	static CTX: OnceLock<Context> = OnceLock::new();
	CTX.get_or_init(|| Context::new(0).unwrap_or_else(|e| panic!("novelpoly-mi355x: no MI355X device ({e:?})")))
}

/// Status code -> the crate's `Error` (errors.rs:4-28, declaration order =
/// codes 1..8); fields from np_last_error_detail.  Codes >= 100 are
/// conditions the crate expresses as panics (asserts) or that only a device
/// can raise: they panic here too.
fn to_error(status: c_int) -> Error {
	let mut d = [0usize; 3];
	unsafe { sys::np_last_error_detail(d.as_mut_ptr()) };
	match status {
		sys::NP_ERR_WANTED_SHARD_COUNT_TOO_HIGH => Error::WantedShardCountTooHigh(d[0]),
		sys::NP_ERR_WANTED_SHARD_COUNT_TOO_LOW => Error::WantedShardCountTooLow(d[0]),
		sys::NP_ERR_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW => Error::WantedPayloadShardCountTooLow(d[0]),
		sys::NP_ERR_PAYLOAD_SIZE_IS_ZERO => Error::PayloadSizeIsZero,
		sys::NP_ERR_NEED_MORE_SHARDS => Error::NeedMoreShards { have: d[0], min: d[1], all: d[2] },
		sys::NP_ERR_PARAMETER_MUST_BE_POWER_OF_2 => Error::ParamterMustBePowerOf2 { n: d[0], k: d[1] },
		sys::NP_ERR_INCONSISTENT_SHARD_LENGTHS => Error::InconsistentShardLengths { first: d[0], other: d[1] },
		sys::NP_ERR_EMPTY_SHARD => Error::EmptyShard,
		s => {
			let msg = unsafe { std::ffi::CStr::from_ptr(sys::np_status_message(s)) };
			// device and allocation failures name the HIP call that returned them
			let site = unsafe { std::ffi::CStr::from_ptr(sys::np_last_error_site()) };
			panic!("novelpoly-mi355x: status {s}: {} [{}]", msg.to_string_lossy(), site.to_string_lossy())
		},
	}
}

fn check(status: c_int) -> Result<()> {
	if status == sys::NP_OK {
		Ok(())
	} else {
		Err(to_error(status))
	}
}

/// `CodeParams` (mod.rs:24-89).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct CodeParams {
	raw: sys::np_code_params,
}

impl CodeParams {
	/// mod.rs:43-61.
	pub fn derive_parameters(n: usize, k: usize) -> Result<CodeParams> {
		let mut raw = sys::np_code_params::default();
		check(unsafe { sys::np_derive_parameters(n, k, &mut raw) })?;
		Ok(CodeParams { raw })
	}

	/// mod.rs:64-71: here, whether a specialised gfx950 kernel serves (n, k).
	pub fn is_faster8(&self) -> bool {
		unsafe { sys::np_is_fast_path(&self.raw) != 0 }
	}

	/// mod.rs:74-77.
	pub fn make_encoder(&self) -> ReedSolomon {
		ReedSolomon { params: *self, ctx: default_context() }
	}

	pub fn make_encoder_on(&self, ctx: &'static Context) -> ReedSolomon {
		ReedSolomon { params: *self, ctx }
	}

	pub fn n(&self) -> usize {
		self.raw.n
	}

	pub fn k(&self) -> usize {
		self.raw.k
	}

	pub fn wanted_n(&self) -> usize {
		self.raw.wanted_n
	}
}

/// `ReedSolomon` (mod.rs:91-285).
pub struct ReedSolomon {
	params: CodeParams,
	ctx: &'static Context,
}

/// Shard pointers and lengths of `received` (None = missing shard).
fn shard_views<S: Shard>(received: &[Option<S>]) -> (Vec<*const u8>, Vec<usize>) {
	let ptrs = received
		.iter()
		.map(|s| s.as_ref().map_or(std::ptr::null(), |s| AsRef::<[u8]>::as_ref(s).as_ptr()))
		.collect();
	let lens = received.iter().map(|s| s.as_ref().map_or(0, |s| AsRef::<[u8]>::as_ref(s).len())).collect();
	(ptrs, lens)
}

impl ReedSolomon {
	/// mod.rs:102-107.
	pub fn shard_len(&self, payload_size: usize) -> usize {
		unsafe { sys::np_shard_len(&self.params.raw, payload_size) }
	}

	/// mod.rs:117-157: `wanted_n` shards of `shard_len(bytes.len())` bytes each.
	pub fn encode<S: Shard>(&self, bytes: &[u8]) -> Result<Vec<S>> {
		if bytes.is_empty() {
			return Err(Error::PayloadSizeIsZero);
		}
		let sl = self.shard_len(bytes.len());
		let mut flat = vec![0u8; self.params.raw.wanted_n * sl];
		check(unsafe {
			sys::np_rs_encode(self.ctx.raw, &self.params.raw, bytes.as_ptr(), bytes.len(), flat.as_mut_ptr(), sl)
		})?;
		Ok(flat.chunks(sl).map(|c| S::from(c.to_vec())).collect())
	}

	/// mod.rs:162-239.  The output is `shard_symbols * 2 * k` bytes (the
	/// payload zero padded), as the crate returns it.
	pub fn reconstruct<S: Shard>(&self, received_shards: Vec<Option<S>>) -> Result<Vec<u8>> {
		let (ptrs, lens) = shard_views(&received_shards);
		let max_syms = lens.iter().map(|l| (l + 1) / 2).max().unwrap_or(0);
		let mut out = vec![0u8; (max_syms * 2 * self.params.raw.k).max(1)];
		let mut out_len = 0usize;
		check(unsafe {
			sys::np_rs_reconstruct(
				self.ctx.raw,
				&self.params.raw,
				ptrs.as_ptr(),
				lens.as_ptr(),
				ptrs.len(),
				out.as_mut_ptr(),
				out.len(),
				&mut out_len,
			)
		})?;
		out.truncate(out_len);
		Ok(out)
	}

	/// mod.rs:247-285: the first k shards, all present.
	pub fn reconstruct_from_systematic<S: Shard>(&self, chunks: Vec<S>) -> Result<Vec<u8>> {
		let ptrs: Vec<*const u8> = chunks.iter().map(|c| AsRef::<[u8]>::as_ref(c).as_ptr()).collect();
		let lens: Vec<usize> = chunks.iter().map(|c| AsRef::<[u8]>::as_ref(c).len()).collect();
		let max_len = lens.iter().copied().max().unwrap_or(0);
		let mut out = vec![0u8; (max_len.div_ceil(2) * 2 * self.params.raw.k).max(1)];
		let mut out_len = 0usize;
		check(unsafe {
			sys::np_rs_reconstruct_from_systematic(
				self.ctx.raw,
				&self.params.raw,
				ptrs.as_ptr(),
				lens.as_ptr(),
				ptrs.len(),
				out.as_mut_ptr(),
				out.len(),
				&mut out_len,
			)
		})?;
		out.truncate(out_len);
		Ok(out)
	}

	/// `batch` payloads of `payload_len` bytes each (payload b at
	/// `payloads[b * payload_len..]`) -> `batch * wanted_n` shards, payload b's
	/// shard v at `out[(b * wanted_n + v) * shard_len..]`.  Equal to calling
	/// `encode` per payload.
	pub fn encode_batch(&self, payloads: &[u8], payload_len: usize) -> Result<Vec<u8>> {
		if payload_len == 0 {
			return Err(Error::PayloadSizeIsZero);
		}
		assert_eq!(payloads.len() % payload_len, 0, "payloads must hold whole payloads");
		let batch = payloads.len() / payload_len;
		let sl = self.shard_len(payload_len);
		let stride = self.params.raw.wanted_n * sl;
		let mut out = vec![0u8; batch * stride];
		check(unsafe {
			sys::np_encode_batch_host(
				self.ctx.raw,
				&self.params.raw,
				payloads.as_ptr(),
				payload_len,
				payload_len,
				batch,
				out.as_mut_ptr(),
				stride,
			)
		})?;
		Ok(out)
	}

	/// `batch` payloads' received rows (payload b's shard v at
	/// `shards[(b * n + v) * shard_len..]`, rows of missing shards ignored) and
	/// their present masks (`present[b * n + v]`) -> each payload's
	/// `shard_len / 2 * 2 * k` bytes.  Equal to calling `reconstruct` per
	/// payload; fails with NeedMoreShards when any payload has fewer than k.
	pub fn reconstruct_batch(&self, shards: &[u8], shard_len: usize, present: &[u8]) -> Result<Vec<u8>> {
		let n = self.params.raw.n;
		assert_eq!(present.len() % n, 0, "present must hold n flags per payload");
		let batch = present.len() / n;
		assert_eq!(shards.len(), batch * n * shard_len, "shards must hold n rows per payload");
		let out_stride = shard_len / 2 * 2 * self.params.raw.k;
		let mut out = vec![0u8; batch * out_stride];
		check(unsafe {
			sys::np_reconstruct_batch_host(
				self.ctx.raw,
				&self.params.raw,
				shards.as_ptr(),
				shard_len,
				n * shard_len,
				present.as_ptr(),
				batch,
				out.as_mut_ptr(),
				out_stride,
			)
		})?;
		Ok(out)
	}
}

/// encode.rs:6-11: derives (n, k) from the validator count like the crate.
pub fn encode<S: Shard>(bytes: &[u8], validator_count: usize) -> Result<Vec<S>> {
	let params = CodeParams::derive_parameters(validator_count, recoverablity_subset_size(validator_count))?;
	params.make_encoder().encode(bytes)
}

/// reconstruct.rs:4-9.
pub fn reconstruct<S: Shard>(received_shards: Vec<Option<S>>, validator_count: usize) -> Result<Vec<u8>> {
	let params = CodeParams::derive_parameters(validator_count, recoverablity_subset_size(validator_count))?;
	params.make_encoder().reconstruct(received_shards)
}

/// util.rs:40.
pub fn recoverablity_subset_size(n_wanted_shards: usize) -> usize {
	unsafe { sys::np_recoverability_subset_size(n_wanted_shards) }
}

/// Several GPUs: one context per device, a batch split into contiguous ranges
/// (np_batch_split), no exchange between devices.
pub struct MultiDevice {
	ctxs: Vec<Context>,
	raws: Vec<*mut sys::np_ctx>,
	lock: Mutex<()>,
}

unsafe impl Send for MultiDevice {}
unsafe impl Sync for MultiDevice {}

impl MultiDevice {
	pub fn new(devices: &[i32]) -> Result<MultiDevice> {
		let ctxs = devices.iter().map(|&d| Context::new(d)).collect::<Result<Vec<_>>>()?;
		let raws = ctxs.iter().map(|c| c.raw).collect();
		Ok(MultiDevice { ctxs, raws, lock: Mutex::new(()) })
	}

	pub fn len(&self) -> usize {
		self.ctxs.len()
	}

	pub fn is_empty(&self) -> bool {
		self.ctxs.is_empty()
	}

	/// As `ReedSolomon::encode_batch`, over every device.
	pub fn encode_batch(&self, params: &CodeParams, payloads: &[u8], payload_len: usize) -> Result<Vec<u8>> {
		if payload_len == 0 {
			return Err(Error::PayloadSizeIsZero);
		}
		assert_eq!(payloads.len() % payload_len, 0, "payloads must hold whole payloads");
		let batch = payloads.len() / payload_len;
		let sl = unsafe { sys::np_shard_len(&params.raw, payload_len) };
		let stride = params.raw.wanted_n * sl;
		let mut out = vec![0u8; batch * stride];
		let _g = self.lock.lock().unwrap();
		check(unsafe {
			sys::np_encode_batch_host_multi(
				self.raws.as_ptr(),
				self.raws.len(),
				&params.raw,
				payloads.as_ptr(),
				payload_len,
				payload_len,
				batch,
				out.as_mut_ptr(),
				stride,
			)
		})?;
		Ok(out)
	}

	/// As `ReedSolomon::reconstruct_batch`, over every device.
	pub fn reconstruct_batch(
		&self,
		params: &CodeParams,
		shards: &[u8],
		shard_len: usize,
		present: &[u8],
	) -> Result<Vec<u8>> {
		let n = params.raw.n;
		assert_eq!(present.len() % n, 0, "present must hold n flags per payload");
		let batch = present.len() / n;
		assert_eq!(shards.len(), batch * n * shard_len, "shards must hold n rows per payload");
		let out_stride = shard_len / 2 * 2 * params.raw.k;
		let mut out = vec![0u8; batch * out_stride];
		let _g = self.lock.lock().unwrap();
		check(unsafe {
			sys::np_reconstruct_batch_host_multi(
				self.raws.as_ptr(),
				self.raws.len(),
				&params.raw,
				shards.as_ptr(),
				shard_len,
				n * shard_len,
				present.as_ptr(),
				batch,
				out.as_mut_ptr(),
				out_stride,
			)
		})?;
		Ok(out)
	}
}

#[cfg(test)]
mod tests {
	//! Bit-exactness against the reference crate itself, shard for shard (the
	//! tests of the repository check the same against the C oracle).
	use super::*;
	use reed_solomon_novelpoly as reference;
	use reference::WrappedShard;

	fn bytes(shards: &[WrappedShard]) -> Vec<Vec<u8>> {
		shards.iter().map(|s| AsRef::<[u8]>::as_ref(s).to_vec()).collect()
	}

	fn payload(len: usize, seed: u64) -> Vec<u8> {
		let mut x = seed.wrapping_mul(0x9E37_79B9_7F4A_7C15) | 1;
		(0..len)
			.map(|_| {
				x ^= x << 13;
				x ^= x >> 7;
				x ^= x << 17;
				x as u8
			})
			.collect()
	}

	#[test]
	fn encode_matches_reference() {
		for &(vc, len) in &[(1024usize, 1 << 20), (256, 12345), (4096, 1 << 19), (2000, 77777), (5, 1)] {
			let p = payload(len, vc as u64);
			let want: Vec<WrappedShard> = reference::encode(&p, vc).unwrap();
			let got: Vec<WrappedShard> = encode(&p, vc).unwrap();
			assert_eq!(bytes(&got), bytes(&want), "vc={vc} len={len}");
		}
	}

	#[test]
	fn reconstruct_matches_reference() {
		for &(vc, len) in &[(1024usize, 1 << 18), (300, 4097), (4096, 1 << 18), (2000, 99999)] {
			let p = payload(len, 7 * vc as u64);
			let shards: Vec<WrappedShard> = reference::encode(&p, vc).unwrap();
			let k = recoverablity_subset_size(vc);
			let received: Vec<Option<WrappedShard>> =
				shards.into_iter().enumerate().map(|(i, s)| if (i * 7919) % vc < k { Some(s) } else { None }).collect();
			let want = reference::reconstruct(received.clone(), vc).unwrap();
			let got = reconstruct(received, vc).unwrap();
			assert_eq!(got, want, "vc={vc}");
			assert_eq!(&got[..len], &p[..]);
		}
	}

	#[test]
	fn errors_match_reference() {
		assert_eq!(encode::<WrappedShard>(&[], 10).unwrap_err(), Error::PayloadSizeIsZero);
		assert_eq!(
			CodeParams::derive_parameters(1, 1).unwrap_err(),
			reference::CodeParams::derive_parameters(1, 1).unwrap_err()
		);
		let shards: Vec<WrappedShard> = encode(&payload(1000, 3), 16).unwrap();
		let received: Vec<Option<WrappedShard>> =
			shards.into_iter().enumerate().map(|(i, s)| if i < 3 { Some(s) } else { None }).collect();
		assert_eq!(
			reconstruct(received.clone(), 16).unwrap_err(),
			reference::reconstruct(received, 16).unwrap_err()
		);
	}
}
