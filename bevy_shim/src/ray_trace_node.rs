//! RayTraceNode (replaces the reference's src/ray_trace_node.rs:16-225).
//! The six compute dispatches become one rt_render call; the result is written
//! into the Rgba32Float texture behind RayTraceOutputImage.
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
use crate::SAMPLES_PER_RAY;

/// Bytes last handed to the tracer (dirty tracking) and the
/// camera block for this frame.
#[derive(Default)]
pub struct SceneUploadState {
    spheres: Vec<u8>,
    materials: Vec<u8>,
    camera: Vec<u8>,
    /// (width, height) the tracer's work buffers were last sized for
    reserved: (u32, u32),
}

/// RenderStage::Prepare, after the reference's own prepare systems have filled
/// ObjectListStorage / MaterialGPUStorage (sphere.rs:180-197,
/// ray_trace_materials.rs:129-164). Uploads the scene only when its packed bytes
/// changed: rt_update_* for a same-size edit, rt_set_scene otherwise.
pub fn prepare_scene(
    ctx: Res<RtContext>,
    camera: Res<RayTraceCamera>,
    objects: Res<ObjectListStorage>,
    materials: Res<MaterialGPUStorage>,
    mut state: ResMut<SceneUploadState>,
) {
    // ObjectListGPU = {u32 sphere_count; pad to 16; N x 32-B SphereGPU} (sphere.rs:19-24)
    let mut sb = encase::StorageBuffer::new(Vec::<u8>::new());
    sb.write(objects.buffer.get()).unwrap();
    let sb = sb.into_inner();
    let n = u32::from_le_bytes([sb[0], sb[1], sb[2], sb[3]]);
    let sph = sb[16..16 + 32 * n as usize].to_vec();
    // Vec<MaterialGPU>: M x 32 B (ray_trace_materials.rs:33-43)
    let mut mb = encase::StorageBuffer::new(Vec::<u8>::new());
    mb.write(materials.buffer.get()).unwrap();
    let mat = mb.into_inner();
    let m = (mat.len() / 32) as u32;

    // CameraGPU exactly as ray_trace_camera.rs:50-63 builds it.
    let t = camera.transform;
    let mut cb = encase::UniformBuffer::new(Vec::<u8>::new());
    cb.write(&CameraGPU {
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
    .unwrap();
    state.camera = cb.into_inner();

    let rc = if state.spheres.len() == sph.len() && state.materials.len() == mat.len()
        && !state.spheres.is_empty()
    {
        let mut rc = 0;
        if let Some((i0, i1)) = dirty_range(&state.materials, &mat, 32) {
            rc = unsafe { rt_update_materials(ctx.0, i0, mat[32 * i0 as usize..].as_ptr() as _, i1 - i0) };
        }
        if rc == 0 {
            if let Some((i0, i1)) = dirty_range(&state.spheres, &sph, 32) {
                rc = unsafe { rt_update_spheres(ctx.0, i0, sph[32 * i0 as usize..].as_ptr() as _, i1 - i0) };
            }
        }
        rc
    } else if sph == state.spheres && mat == state.materials {
        0
    } else {
        unsafe { rt_set_scene(ctx.0, sph.as_ptr() as _, n, mat.as_ptr() as _, m) }
    };
    match ctx.check(rc) {
        Ok(()) => {
            state.spheres = sph;
            state.materials = mat;
        }
        Err(e) => error!("scene upload: {e}"),
    }

    // Size the frame's work buffers here, not inside RayTraceNode::run, as the
    // reference re-sizes its ray buffers in prepare (ray_trace_rays.rs:50-66).
    let size = (camera.render_width, camera.render_height);
    if size != state.reserved {
        let params = rt_params {
            width: size.0,
            height: size.1,
            spp: SAMPLES_PER_RAY as u32,
            max_depth: 3, // ray_trace_node.rs:213
            row_block: 8,
            shard_count: 1,
            ..Default::default()
        };
        match ctx.check(unsafe { rt_reserve(ctx.0, &params, 1) }) {
            Ok(()) => state.reserved = size,
            Err(e) => error!("rt_reserve: {e}"),
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

#[derive(Default)]
pub struct RayTraceNode {
    texels: std::sync::Mutex<Vec<f32>>,
}

impl render_graph::Node for RayTraceNode {
    fn update(&mut self, _world: &mut World) {}

    fn run(
        &self,
        _graph: &mut RenderGraphContext,
        _render_context: &mut RenderContext,
        world: &World,
    ) -> Result<(), NodeRunError> {
        let ctx = world.resource::<RtContext>();
        let state = world.resource::<SceneUploadState>();
        let camera = world.resource::<RayTraceCamera>();
        // frame = RNG seed input (ray_trace_globals.rs:56-68)
        let frame = world.resource::<GlobalsGPUStorage>().buffer.get().frame;

        let (w, h) = (camera.render_width, camera.render_height);
        let params = rt_params {
            width: w,
            height: h,
            spp: SAMPLES_PER_RAY as u32,
            max_depth: 3, // ray_trace_node.rs:213
            frame0: frame,
            row_block: 8,
            shard_count: 1,
            ..Default::default()
        };
        let mut texels = self.texels.lock().unwrap();
        texels.resize((w * h * 4) as usize, 0.0);
        let rc = unsafe {
            rt_render(ctx.0, state.camera.as_ptr() as _, &params, texels.as_mut_ptr(),
                      std::ptr::null_mut())
        };
        if let Err(e) = ctx.check(rc) {
            error!("rt_render: {e}"); // keep showing the previous frame
            return Ok(());
        }
        let images = world.resource::<RenderAssets<Image>>();
        let output = &images[&world.resource::<RayTraceOutputImage>().0];
        world.resource::<RenderQueue>().write_texture(
            output.texture.as_image_copy(),
            bytemuck::cast_slice(&texels[..]),
            ImageDataLayout {
                offset: 0,
                bytes_per_row: NonZeroU32::new(w * 16),
                rows_per_image: None,
            },
            Extent3d { width: w, height: h, depth_or_array_layers: 1 },
        );
        Ok(())
    }
}
