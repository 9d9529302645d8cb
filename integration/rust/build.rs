// build.rs addition for the reference crate: link libmarshrutka_pf.so, built by
// `python -m marshrutka_amd.build` into <repo>/marshrutka_amd/lib.  MARSHRUTKA_PF_LIB
// overrides the directory.
fn main() {
    let dir = std::env::var("MARSHRUTKA_PF_LIB").unwrap_or_else(|_| "../marshrutka_amd/lib".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=marshrutka_pf");
    println!("cargo:rerun-if-env-changed=MARSHRUTKA_PF_LIB");
}
