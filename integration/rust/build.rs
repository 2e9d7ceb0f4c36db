// UNVERIFIED (no cargo here).  Builds libdchess.so for gfx950 with the repo's
// Makefile (hipcc --offload-arch=gfx950) and links it; see INTEGRATION.md §2.
fn main() {
    let root = std::path::PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap()).join("../..");
    let pkg = root.join("distributed-chess_amd");
    let ok = std::process::Command::new("make")
        .args(["-C", pkg.to_str().unwrap(), "libdchess.so"])
        .env("ARCH", "gfx950")
        .status()
        .expect("make");
    assert!(ok.success(), "hipcc build of libdchess.so failed");
    println!("cargo:rustc-link-search=native={}", pkg.display());
    println!("cargo:rustc-link-lib=dylib=dchess");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", pkg.display());
    println!("cargo:rerun-if-changed={}", pkg.join("csrc").display());
    println!("cargo:rerun-if-changed={}", root.join("include/dchess.h").display());
}
