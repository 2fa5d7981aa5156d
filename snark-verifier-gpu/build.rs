//! Links libsvgpu.so, built by `make -C snark-verifier-axiom_amd` (hipcc --offload-arch=gfx950).
//! SVGPU_LIB_DIR overrides the search directory (default: the in-tree build next to this crate).
fn main() {
    let dir = std::env::var("SVGPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{here}/../snark-verifier-axiom_amd/build")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=svgpu");
    println!("cargo:rerun-if-env-changed=SVGPU_LIB_DIR");
    println!("cargo:rerun-if-changed=../include/svgpu.h");
}
