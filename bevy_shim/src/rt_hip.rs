//! FFI for include/rt_hip.h (the MI355X path tracer's C-ABI).
#![allow(non_camel_case_types, dead_code)]
use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
pub struct rt_ctx {
    _private: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct rt_params {
    pub width: u32,
    pub height: u32,
    pub spp: u32,
    pub max_depth: u32,
    pub frame0: u32,
    pub row_block: u32,
    pub shard_count: u32,
    pub shard_index: u32,
    pub flags: u32,
    pub _reserved: [u32; 3],
}

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct rt_stats {
    pub segments: u64,
    pub traced_segments: u64,
    pub sphere_tests: u64,
    pub paths: u64,
    pub kernel_ms: f64,
    pub total_ms: f64,
    pub kernel_launches: u32,
    pub short_math: u32,
    pub clock_ghz: f64,
}

/// Renders that may be in flight on one context (rt_hip.h RT_MAX_PENDING).
pub const RT_MAX_PENDING: u32 = 2;
pub const RT_FLAG_NO_PRIMARY_CACHE: u32 = 0x1;
/// Opt-in camera sampling (rt_hip.h): sub-pixel jitter and thin-lens samples
/// through the reference's thin_lens_ray (generate.wgsl:85-107).
pub const RT_FLAG_JITTER: u32 = 0x2;
pub const RT_FLAG_THIN_LENS: u32 = 0x4;
/// Culled sphere list: identical hits, less filter work (rt_hip.h).
pub const RT_FLAG_CULL: u32 = 0x8;
/// The packed-fp32 VALU filter instead of the matrix-core one: identical hits
/// (rt_hip.h; A/B and cross-checks).
pub const RT_FLAG_VALU_FILTER: u32 = 0x10;
/// Device-output calls write whole images: the owned rows at their image rows.
pub const RT_FLAG_IMAGE_OUT: u32 = 0x20;

extern "C" {
    pub fn rt_version() -> c_int;
    pub fn rt_create(device: c_int, out_ctx: *mut *mut rt_ctx) -> c_int;
    pub fn rt_destroy(ctx: *mut rt_ctx);
    pub fn rt_set_scene(ctx: *mut rt_ctx, spheres: *const c_void, n: u32,
                        materials: *const c_void, m: u32) -> c_int;
    pub fn rt_update_spheres(ctx: *mut rt_ctx, first: u32, spheres: *const c_void, count: u32) -> c_int;
    pub fn rt_update_materials(ctx: *mut rt_ctx, first: u32, materials: *const c_void, count: u32) -> c_int;
    pub fn rt_render(ctx: *mut rt_ctx, camera: *const c_void, params: *const rt_params,
                     out_rgba: *mut f32, stats: *mut rt_stats) -> c_int;
    pub fn rt_render_progressive(ctx: *mut rt_ctx, camera: *const c_void, params: *const rt_params,
                                 reset: c_int, out_rgba: *mut f32, total_spp: *mut u64) -> c_int;
    // nframes consecutive frames (frame i = samples frame0 + i*spp ...) in one
    // persistent launch, into device memory; complete with rt_wait
    pub fn rt_render_frames_device(ctx: *mut rt_ctx, camera: *const c_void, params: *const rt_params,
                                   nframes: u32, out_rgba_device: *mut f32,
                                   stream: *mut c_void) -> c_int;
    // allocate a launch's work buffers up front (RayTraceNode setup, not run)
    pub fn rt_reserve(ctx: *mut rt_ctx, params: *const rt_params, nframes: u32) -> c_int;
    // enqueue a frame into a HOST buffer; rt_wait completes it (copy + stats)
    pub fn rt_render_async(ctx: *mut rt_ctx, camera: *const c_void, params: *const rt_params,
                           out_rgba: *mut f32) -> c_int;
    pub fn rt_wait(ctx: *mut rt_ctx, stats: *mut rt_stats) -> c_int;
    // page-lock a host buffer rt_render_async writes: its copy is then a DMA
    // and rt_render_async returns at once (pageable: it waits for the frame)
    pub fn rt_host_register(ctx: *mut rt_ctx, ptr: *mut c_void, bytes: usize) -> c_int;
    pub fn rt_host_unregister(ctx: *mut rt_ctx, ptr: *mut c_void) -> c_int;
    pub fn rt_intersect(ctx: *mut rt_ctx, rays: *const f32, n: u32, hit_index: *mut i32,
                        hit_t: *mut f32) -> c_int;
    // multi-GPU only: system-scope acquire on the image owner's device
    // before it reads rows other ranks wrote with RT_FLAG_IMAGE_OUT
    pub fn rt_acquire(ctx: *mut rt_ctx, stream: *mut c_void) -> c_int;
    pub fn rt_last_error(ctx: *const rt_ctx) -> *const c_char;
}

/// Owner of one rt_ctx (one per GPU). Calls are serialised by the render thread.
pub struct RtContext(pub *mut rt_ctx);
unsafe impl Send for RtContext {}
unsafe impl Sync for RtContext {}

impl RtContext {
    pub fn new(device: i32) -> Result<Self, String> {
        let mut ctx = std::ptr::null_mut();
        let rc = unsafe { rt_create(device, &mut ctx) };
        if rc != 0 {
            return Err(last_error(std::ptr::null()));
        }
        Ok(RtContext(ctx))
    }
    pub fn check(&self, rc: c_int) -> Result<(), String> {
        if rc == 0 { Ok(()) } else { Err(last_error(self.0)) }
    }
}

impl Drop for RtContext {
    fn drop(&mut self) {
        unsafe { rt_destroy(self.0) }
    }
}

pub fn last_error(ctx: *const rt_ctx) -> String {
    unsafe { CStr::from_ptr(rt_last_error(ctx)).to_string_lossy().into_owned() }
}
