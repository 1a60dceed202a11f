// Links libstratum_hip.so, built by `make -C stratum-dsp_amd` (HIP, gfx950).  Set
// STRATUM_HIP_LIB_DIR to its directory (default: ../stratum-dsp_amd/lib next to this crate).
fn main() {
    let dir = std::env::var("STRATUM_HIP_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{here}/../stratum-dsp_amd/lib")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=stratum_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=STRATUM_HIP_LIB_DIR");
}
