//! RayTracePlugin (replaces the reference's src/plugin.rs:19-122): same name,
//! same sub-plugins for the camera / globals / materials / output resources,
//! but no wgpu pipelines or bind groups -- the render-graph node calls the
//! MI355X path tracer through the C-ABI.
use bevy::{
    prelude::*,
    render::{render_graph::RenderGraph, RenderApp, RenderStage},
};

use crate::ray_trace_camera::RayTraceCameraPlugin;
use crate::ray_trace_globals::RayTraceGlobalsPlugin;
use crate::ray_trace_materials::RayTraceMaterialsPlugin;
use crate::ray_trace_node::{prepare_scene, RayTraceNode, SceneUploadState};
use crate::ray_trace_output::RayTraceOutputPlugin;
use crate::rt_hip::RtContext;

pub struct RayTracePlugin;

impl Plugin for RayTracePlugin {
    fn build(&self, app: &mut App) {
        app.add_plugin(RayTraceCameraPlugin)
            .add_plugin(RayTraceGlobalsPlugin)
            .add_plugin(RayTraceMaterialsPlugin)
            .add_plugin(RayTraceOutputPlugin);

        let render_app = app.sub_app_mut(RenderApp);
        let ctx = RtContext::new(0).expect("rt_create failed (no MI355X / librt_hip.so?)");
        render_app
            .insert_resource(ctx)
            .init_resource::<SceneUploadState>()
            // after sphere.rs / ray_trace_materials.rs `prepare` have packed the bytes
            .add_system_to_stage(RenderStage::Prepare, prepare_scene.at_end());

        let mut render_graph = render_app.world.resource_mut::<RenderGraph>();
        render_graph.add_node("raytrace", RayTraceNode::default());
        render_graph
            .add_node_edge("raytrace", bevy::render::main_graph::node::CAMERA_DRIVER)
            .unwrap();
    }
}
