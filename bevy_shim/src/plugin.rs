//! RayTracePlugin (replaces the reference's src/plugin.rs:19-122): same name,
//! same sub-plugins for the camera / globals / materials / output resources,
//! but no wgpu pipelines or bind groups -- the render-graph node calls the
//! MI355X path tracer through the C-ABI (include/rt_hip.h).
use bevy::{
    prelude::*,
    render::{render_graph::RenderGraph, RenderApp},
};

use crate::ray_trace_camera::RayTraceCameraPlugin;
use crate::ray_trace_globals::RayTraceGlobalsPlugin;
use crate::ray_trace_materials::RayTraceMaterialsPlugin;
use crate::ray_trace_node::RayTraceNode;
use crate::ray_trace_output::RayTraceOutputPlugin;
use crate::rt_hip::RtContext;

pub struct RayTracePlugin;

impl Plugin for RayTracePlugin {
    fn build(&self, app: &mut App) {
        app.add_plugin(RayTraceCameraPlugin)
            .add_plugin(RayTraceGlobalsPlugin)
            .add_plugin(RayTraceMaterialsPlugin)
            .add_plugin(RayTraceOutputPlugin);

        // One context on HIP device 0. Without a device (or librt_hip.so's
        // kernels) the app keeps running with the cleared output image, like
        // the reference while its pipelines are still loading
        // (ray_trace_node.rs:201-202): the error is logged, nothing panics.
        let ctx = match RtContext::new(0) {
            Ok(ctx) => ctx,
            Err(e) => {
                error!("RayTracePlugin: rt_create failed, ray tracing disabled: {e}");
                return;
            }
        };
        let render_app = app.sub_app_mut(RenderApp);
        let mut render_graph = render_app.world.resource_mut::<RenderGraph>();
        // the node owns the context: rt_destroy runs when the render graph drops it
        render_graph.add_node("raytrace", RayTraceNode::new(ctx));
        if let Err(e) =
            render_graph.add_node_edge("raytrace", bevy::render::main_graph::node::CAMERA_DRIVER)
        {
            error!("RayTracePlugin: render graph edge: {e:?}");
        }
    }
}
