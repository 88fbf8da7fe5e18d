//! Links libnovelpoly_hip.so, built by `make -C reed-solomon-novelpoly_amd`
//! (gfx950).  NOVELPOLY_MI355X_LIB names the directory holding it; default:
//! the in-tree build output of this repository.
fn main() {
	let dir = std::env::var("NOVELPOLY_MI355X_LIB").unwrap_or_else(|_| {
		let here = std::env::var("CARGO_MANIFEST_DIR").expect("cargo sets CARGO_MANIFEST_DIR");
		format!("{here}/../../../reed-solomon-novelpoly_amd/lib")
	});
	println!("cargo:rustc-link-search=native={dir}");
	println!("cargo:rustc-link-lib=dylib=novelpoly_hip");
	println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
	println!("cargo:rerun-if-env-changed=NOVELPOLY_MI355X_LIB");
}
