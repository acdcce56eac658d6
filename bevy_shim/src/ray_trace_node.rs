//! RayTraceNode (replaces the reference's src/ray_trace_node.rs:16-225).
//! The reference's six compute dispatches become one rt_render_async call on
//! the MI355X; the finished Rgba32Float frame is written into the texture
//! behind RayTraceOutputImage.
//!
//! Per frame, in `update` (it has `&mut World`, runs after every RenderStage
//! ::Prepare system, so sphere.rs / ray_trace_materials.rs / ray_trace_globals.rs
//! have packed this frame's bytes):
//!   1. with `frames_in_flight` renders pending (1 by default, at most
//!      RT_MAX_PENDING = 2), rt_wait for the oldest -- its texels become the
//!      frame `run` shows;
//!   2. dirty-tracked scene upload: rt_update_* for a same-size edit,
//!      rt_set_scene when the counts change, nothing when the bytes are equal
//!      (the reference re-uploads everything every frame, sphere.rs:180-197);
//!   3. rt_reserve when the output size changes (the reference sizes its
//!      buffers in prepare, ray_trace_rays.rs:50-66, not in run; it needs no
//!      render in flight, so a resize first completes the pending ones);
//!   4. rt_render_async of this frame into a host buffer that is neither shown
//!      nor in flight (three buffers).
//! Frames in flight (`RayTraceNode::with_frames_in_flight`): with 1 (the
//! default, `new`) the frame enqueued in one update is shown by the next --
//! one frame of latency, as the round-3 shim; with 2 each pending frame has
//! its own stream in the library, so frame n's device->host copy overlaps
//! frame n+1's render (the copy is 45 % of a 1080p frame at 1 spp,
//! profiles/r03_bench_reference1080.json; bench.py shim_sequence measures
//! both depths: 697 vs 1,365 frames/s) at the price of one more frame of
//! input latency (the shown frame is two behind the camera). `run` only
//! copies the finished frame into the texture. A failing call is logged and
//! skipped (the previous image stays); nothing panics across the render
//! thread.
use std::num::NonZeroU32;

use bevy::{
    prelude::*,
    render::{
        render_asset::RenderAssets,
        render_graph::{self, NodeRunError, RenderGraphContext},
        render_resource::{encase, *},
        renderer::{RenderContext, RenderQueue},
    },
};

use crate::camera::RayTraceCamera;
use crate::ray_trace_camera::CameraGPU;
use crate::ray_trace_globals::GlobalsGPUStorage;
use crate::ray_trace_materials::MaterialGPUStorage;
use crate::ray_trace_output::RayTraceOutputImage;
use crate::rt_hip::*;
use crate::sphere::ObjectListStorage;
use crate::{RENDER_TARGET_SIZE, SAMPLES_PER_RAY};

/// The reference's loop count of (prepass, intersect, shade), ray_trace_node.rs:213.
const MAX_DEPTH: u32 = 3;

/// Bytes last handed to the tracer (dirty tracking).
#[derive(Default)]
struct Uploaded {
    spheres: Vec<u8>,
    materials: Vec<u8>,
    /// the tracer holds exactly these bytes (false: upload in full)
    scene_ok: bool,
    /// (width, height) the work buffers were last reserved for
    reserved: (u32, u32),
}

/// One host frame buffer and the geometry it holds.
#[derive(Default)]
struct HostFrame {
    texels: Vec<f32>,
    size: (u32, u32),
    /// texels' (pointer, length) as given to rt_host_register, if registered
    registered: Option<(usize, usize)>,
}

/// Host frame buffers: the shown one and up to RT_MAX_PENDING in flight
/// (with fewer frames in flight the last ones are never allocated).
const NBUF: usize = RT_MAX_PENDING as usize + 1;

pub struct RayTraceNode {
    ctx: RtContext,
    uploaded: Uploaded,
    camera: Vec<u8>,
    frames: [HostFrame; NBUF],
    /// buffers rt_render_async calls are pending into, oldest first
    pending: std::collections::VecDeque<usize>,
    /// index of the last finished frame (what `run` shows)
    ready: Option<usize>,
    /// renders kept in flight across updates, 1..=RT_MAX_PENDING
    frames_in_flight: usize,
}

impl RayTraceNode {
    /// One render in flight: the frame enqueued in an update is shown by the
    /// next one (one frame of latency).
    pub fn new(ctx: RtContext) -> Self {
        Self::with_frames_in_flight(ctx, 1)
    }

    /// `depth` renders in flight (clamped to 1..=RT_MAX_PENDING): 2 overlaps a
    /// frame's device->host copy with the next render (about twice the frame
    /// rate at 1 spp) and shows frames two behind the camera.
    pub fn with_frames_in_flight(ctx: RtContext, depth: u32) -> Self {
        RayTraceNode {
            ctx,
            uploaded: Uploaded::default(),
            camera: Vec::new(),
            frames: Default::default(),
            pending: std::collections::VecDeque::new(),
            ready: None,
            frames_in_flight: depth.clamp(1, RT_MAX_PENDING) as usize,
        }
    }

    fn params(&self, size: (u32, u32), frame: u32) -> rt_params {
        rt_params {
            width: size.0,
            height: size.1,
            spp: SAMPLES_PER_RAY as u32,
            max_depth: MAX_DEPTH,
            frame0: frame,
            row_block: 8,
            shard_count: 1,
            // the brute-force walk (matrix-core filter): on the reference's
            // own frame (1920x1080, 1 spp, depth 3, its dim-7 scene) it is
            // faster than the culled list, 0.66 vs 0.80 ms of kernel per
            // frame (profiles/r03_bench_reference1080.json: shim_sequence)
            flags: 0,
            ..Default::default()
        }
    }

    /// Complete the oldest render in flight (rt_wait completes the oldest).
    fn finish_oldest(&mut self) {
        if let Some(i) = self.pending.pop_front() {
            let mut st = rt_stats::default();
            match self.ctx.check(unsafe { rt_wait(self.ctx.0, &mut st) }) {
                Ok(()) => self.ready = Some(i),
                Err(e) => error!("rt_wait: {e}"),
            }
        }
    }

    /// Step 1: keep at most frames_in_flight - 1 renders in flight before
    /// enqueueing this frame's.
    fn finish_pending(&mut self) {
        while self.pending.len() >= self.frames_in_flight {
            self.finish_oldest();
        }
    }

    /// Every render in flight (before rt_reserve, and on drop).
    fn finish_all(&mut self) {
        while !self.pending.is_empty() {
            self.finish_oldest();
        }
    }

    /// Step 2: the scene, only when its packed bytes changed.
    fn upload_scene(&mut self, world: &World) {
        // ObjectListGPU = {u32 sphere_count; pad to 16; N x 32-B SphereGPU} (sphere.rs:19-24)
        let mut sb = encase::StorageBuffer::new(Vec::<u8>::new());
        if sb.write(world.resource::<ObjectListStorage>().buffer.get()).is_err() {
            error!("scene upload: cannot pack the sphere list");
            return;
        }
        let sb = sb.into_inner();
        let n = u32::from_le_bytes([sb[0], sb[1], sb[2], sb[3]]);
        let sph = sb[16..16 + 32 * n as usize].to_vec();
        // Vec<MaterialGPU>: M x 32 B (ray_trace_materials.rs:33-43)
        let mut mb = encase::StorageBuffer::new(Vec::<u8>::new());
        if mb.write(world.resource::<MaterialGPUStorage>().buffer.get()).is_err() {
            error!("scene upload: cannot pack the materials");
            return;
        }
        let mat = mb.into_inner();
        let m = (mat.len() / 32) as u32;
        let (old_s, old_m) = (&self.uploaded.spheres, &self.uploaded.materials);
        let ok = self.uploaded.scene_ok;
        if ok && sph == *old_s && mat == *old_m {
            return;
        }
        let ctx = self.ctx.0;
        let rc = if ok && old_s.len() == sph.len() && old_m.len() == mat.len() {
            let mut rc = 0;
            if let Some((i0, i1)) = dirty_range(old_m, &mat, 32) {
                let p = mat[32 * i0 as usize..].as_ptr() as *const _;
                rc = unsafe { rt_update_materials(ctx, i0, p, i1 - i0) };
            }
            if rc == 0 {
                if let Some((i0, i1)) = dirty_range(old_s, &sph, 32) {
                    let p = sph[32 * i0 as usize..].as_ptr() as *const _;
                    rc = unsafe { rt_update_spheres(ctx, i0, p, i1 - i0) };
                }
            }
            rc
        } else {
            unsafe { rt_set_scene(ctx, sph.as_ptr() as *const _, n, mat.as_ptr() as *const _, m) }
        };
        match self.ctx.check(rc) {
            Ok(()) => {
                self.uploaded.spheres = sph;
                self.uploaded.materials = mat;
                self.uploaded.scene_ok = true;
            }
            Err(e) => {
                // a failed rt_set_scene leaves no scene: upload in full next frame
                self.uploaded = Uploaded::default();
                error!("scene upload: {e}");
            }
        }
    }

    /// CameraGPU exactly as ray_trace_camera.rs:50-63 packs it (std140, 128 B).
    fn pack_camera(&mut self, camera: &RayTraceCamera) {
        let t = camera.transform;
        let mut cb = encase::UniformBuffer::new(Vec::<u8>::new());
        let ok = cb
            .write(&CameraGPU {
                transform: t.compute_matrix(),
                forward: t.forward(),
                up: t.up(),
                right: t.right(),
                position: t.translation,
                fov: 1.5708,
                image_plane_distance: 10.0,
                lens_focal_length: 0.1,
                fstop: 1.0 / 32.0,
            })
            .is_ok();
        if ok {
            self.camera = cb.into_inner();
        }
    }
}

/// [first, last+1) of the records that differ, or None.
fn dirty_range(old: &[u8], new: &[u8], rec: usize) -> Option<(u32, u32)> {
    let mut lo = None;
    let mut hi = 0;
    for (i, (a, b)) in old.chunks(rec).zip(new.chunks(rec)).enumerate() {
        if a != b {
            lo.get_or_insert(i);
            hi = i + 1;
        }
    }
    lo.map(|l| (l as u32, hi as u32))
}

impl render_graph::Node for RayTraceNode {
    fn update(&mut self, world: &mut World) {
        self.finish_pending();
        self.upload_scene(world);
        if !self.uploaded.scene_ok {
            return; // no scene on the device: nothing to render
        }
        let camera = world.resource::<RayTraceCamera>().clone();
        self.pack_camera(&camera);
        if self.camera.len() != 128 {
            return;
        }
        let size = (camera.render_width, camera.render_height);
        // seed frame (ray_trace_globals.rs:56-68)
        let frame = world.resource::<GlobalsGPUStorage>().buffer.get().frame;
        let params = self.params(size, frame);
        if size != self.uploaded.reserved {
            self.finish_all(); // rt_reserve requires no render in flight
            match self.ctx.check(unsafe { rt_reserve(self.ctx.0, &params, 1) }) {
                Ok(()) => self.uploaded.reserved = size,
                Err(e) => error!("rt_reserve: {e}"),
            }
        }
        // a buffer `run` does not show and no render is pending into
        let i = match (0..NBUF).find(|b| Some(*b) != self.ready && !self.pending.contains(b)) {
            Some(i) => i,
            None => return,
        };
        let buf = &mut self.frames[i];
        let len = (size.0 * size.1 * 4) as usize;
        if buf.texels.len() != len {
            // resize() may move the allocation: unregister the old one first,
            // while it is still ours (no render is pending into this buffer)
            if let Some((p, _)) = buf.registered.take() {
                let _ = self.ctx.check(unsafe { rt_host_unregister(self.ctx.0, p as *mut _) });
            }
            buf.texels.resize(len, 0.0);
        }
        buf.size = size;
        // page-locked once per allocation: the device->host copy is then a DMA
        // and rt_render_async returns at once instead of waiting for the frame
        // (1.32 vs 0.03 ms per call at 1080p, profiles/r03_bench_reference1080.json)
        let key = (buf.texels.as_ptr() as usize, buf.texels.len());
        if buf.registered != Some(key) {
            if let Some((p, _)) = buf.registered.take() {
                let _ = self.ctx.check(unsafe { rt_host_unregister(self.ctx.0, p as *mut _) });
            }
            let bytes = buf.texels.len() * std::mem::size_of::<f32>();
            match self.ctx.check(unsafe {
                rt_host_register(self.ctx.0, buf.texels.as_mut_ptr() as *mut _, bytes)
            }) {
                Ok(()) => buf.registered = Some(key),
                Err(e) => error!("rt_host_register: {e}"),
            }
        }
        let rc = unsafe {
            rt_render_async(self.ctx.0, self.camera.as_ptr() as *const _, &params,
                            buf.texels.as_mut_ptr())
        };
        match self.ctx.check(rc) {
            Ok(()) => self.pending.push_back(i),
            Err(e) => error!("rt_render_async: {e}"),
        }
    }

    fn run(
        &self,
        _graph: &mut RenderGraphContext,
        _render_context: &mut RenderContext,
        world: &World,
    ) -> Result<(), NodeRunError> {
        let f = match self.ready {
            Some(i) => &self.frames[i],
            None => return Ok(()),
        };
        // the target is created at RENDER_TARGET_SIZE (ray_trace_output.rs init_output)
        if f.size != RENDER_TARGET_SIZE {
            return Ok(());
        }
        let images = world.resource::<RenderAssets<Image>>();
        let output = match images.get(&world.resource::<RayTraceOutputImage>().0) {
            Some(o) => o,
            None => return Ok(()), // not prepared yet
        };
        world.resource::<RenderQueue>().write_texture(
            output.texture.as_image_copy(),
            bytemuck::cast_slice(&f.texels[..]),
            ImageDataLayout {
                offset: 0,
                bytes_per_row: NonZeroU32::new(f.size.0 * 16),
                rows_per_image: None,
            },
            Extent3d { width: f.size.0, height: f.size.1, depth_or_array_layers: 1 },
        );
        Ok(())
    }
}

impl Drop for RayTraceNode {
    fn drop(&mut self) {
        // the host buffers of pending renders must outlive them
        self.finish_all();
        // self.ctx drops next: rt_destroy
    }
}
