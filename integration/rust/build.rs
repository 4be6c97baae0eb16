// Links librs_simplify.so (built in-tree by circom_cvm_amd/build.py: hipcc --offload-arch=gfx950).
fn main() {
    let dir = std::env::var("RS_SIMPLIFY_LIB_DIR").unwrap_or_else(|_| "../../circom_cvm_amd".to_string());
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-lib=dylib=rs_simplify");
    println!("cargo:rerun-if-env-changed=RS_SIMPLIFY_LIB_DIR");
}
