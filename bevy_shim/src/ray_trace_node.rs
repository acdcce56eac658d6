//! RayTraceNode (replaces the reference's src/ray_trace_node.rs:16-225).
//! The six compute dispatches become one rt_render call; the result is written
//! into the Rgba32Float texture behind RayTraceOutputImage.
use std::num::NonZeroU32;

use bevy::{
    prelude::*,
    render::{
        render_asset::RenderAssets,
        render_graph::{self, NodeRunError, RenderGraphContext},
        render_resource::*,
        renderer::{RenderContext, RenderQueue},
    },
};

use crate::ray_trace_camera::CameraGPUStorage;
use crate::ray_trace_globals::GlobalsGPU;
use crate::ray_trace_materials::MaterialGPUStorage;
use crate::ray_trace_output::RayTraceOutputImage;
use crate::rt_hip::*;
use crate::sphere::ObjectListStorage;
use crate::{RENDER_TARGET_SIZE, SAMPLES_PER_RAY};

/// Bytes last uploaded with rt_set_scene (dirty tracking).
#[derive(Default)]
pub struct SceneUploadState {
    spheres: Vec<u8>,
    materials: Vec<u8>,
}

/// RenderStage::Prepare: upload the scene only when its packed bytes changed.
/// ObjectListGPU = {u32 count; pad to 16; N x 32-B SphereGPU} (sphere.rs:19-24).
pub fn prepare_scene(
    ctx: Res<RtContext>,
    objects: Res<ObjectListStorage>,
    materials: Res<MaterialGPUStorage>,
    mut state: ResMut<SceneUploadState>,
) {
    let obj = objects.buffer.get();
    let mut sbytes = encase::StorageBuffer::new(Vec::<u8>::new());
    sbytes.write(obj).unwrap();
    let sbytes = sbytes.into_inner();
    let mut mbytes = encase::StorageBuffer::new(Vec::<u8>::new());
    mbytes.write(materials.buffer.get()).unwrap();
    let mbytes = mbytes.into_inner();
    if sbytes == state.spheres && mbytes == state.materials {
        return;
    }
    let n = obj.sphere_count;
    let m = (mbytes.len() / 32) as u32;
    let rc = unsafe {
        rt_set_scene(ctx.0, sbytes[16..].as_ptr() as *const _, n, mbytes.as_ptr() as *const _, m)
    };
    if let Err(e) = ctx.check(rc) {
        error!("rt_set_scene: {e}");
        return;
    }
    state.spheres = sbytes;
    state.materials = mbytes;
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
        let globals = world.resource::<GlobalsGPU>(); // frame = RNG seed input
        let camera = world.resource::<CameraGPUStorage>();
        let mut cam = encase::UniformBuffer::new(Vec::<u8>::new());
        cam.write(&camera.current()).unwrap(); // the 128-B std140 CameraGPU block
        let cam = cam.into_inner();

        let (w, h) = RENDER_TARGET_SIZE;
        let params = rt_params {
            width: w,
            height: h,
            spp: SAMPLES_PER_RAY as u32,
            max_depth: 3, // ray_trace_node.rs:213
            frame0: globals.frame,
            row_block: 8,
            shard_count: 1,
            ..Default::default()
        };
        let mut texels = self.texels.lock().unwrap();
        texels.resize((w * h * 4) as usize, 0.0);
        let rc = unsafe {
            rt_render(ctx.0, cam.as_ptr() as *const _, &params, texels.as_mut_ptr(),
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
