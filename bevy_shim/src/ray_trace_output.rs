//! RayTraceOutputImage and its sprite (replaces the reference's
//! src/ray_trace_output.rs). What stays: the Rgba32Float render target of
//! RENDER_TARGET_SIZE shown through a sprite, extracted to the render world,
//! and the sprite following window resizes (ray_trace_output.rs:19-97 there).
//! What goes: the storage-texture bind group built in RenderStage::Queue from
//! `RayTracePipeline`'s layout (ray_trace_output.rs:99-117, `describe`
//! 121-136) -- the pipeline no longer exists; RayTraceNode writes the frame
//! into the texture with RenderQueue::write_texture, which needs COPY_DST.
use bevy::{
    prelude::*,
    render::{
        extract_resource::{ExtractResource, ExtractResourcePlugin},
        render_resource::{Extent3d, TextureDimension, TextureFormat, TextureUsages},
    },
    window::WindowResized,
};

use crate::RENDER_TARGET_SIZE;

/// Marks the sprite entity that displays the ray-traced image.
#[derive(Component)]
pub struct RenderTarget;

/// Handle of the output image (the field is public: RayTraceNode reads it
/// in the render world).
#[derive(Clone, Deref, ExtractResource)]
pub struct RayTraceOutputImage(pub Handle<Image>);

pub struct RayTraceOutputPlugin;

impl Plugin for RayTraceOutputPlugin {
    fn build(&self, app: &mut App) {
        app.add_plugin(ExtractResourcePlugin::<RayTraceOutputImage>::default())
            .add_startup_system(create_output_image)
            .add_system(fit_sprite_to_window);
    }
}

/// The render target, cleared to opaque black, and a sprite of the same size
/// that shows it.
fn create_output_image(mut commands: Commands, mut images: ResMut<Assets<Image>>) {
    let (w, h) = RENDER_TARGET_SIZE;
    let black: [f32; 4] = [0.0, 0.0, 0.0, 1.0];
    let mut image = Image::new_fill(
        Extent3d { width: w, height: h, depth_or_array_layers: 1 },
        TextureDimension::D2,
        bytemuck::cast_slice(&black),
        TextureFormat::Rgba32Float,
    );
    // written by RenderQueue::write_texture, sampled by the sprite pass
    image.texture_descriptor.usage = TextureUsages::COPY_DST | TextureUsages::TEXTURE_BINDING;
    let handle = images.add(image);
    commands
        .spawn_bundle(SpriteBundle {
            sprite: Sprite { custom_size: Some(Vec2::new(w as f32, h as f32)), ..default() },
            texture: handle.clone(),
            ..default()
        })
        .insert(RenderTarget);
    commands.insert_resource(RayTraceOutputImage(handle));
}

/// Stretch the sprite over the window after a resize (the render target
/// keeps its size).
fn fit_sprite_to_window(
    mut resized: EventReader<WindowResized>,
    mut sprites: Query<&mut Sprite, With<RenderTarget>>,
) {
    if let Some(e) = resized.iter().last() {
        for mut sprite in sprites.iter_mut() {
            sprite.custom_size = Some(Vec2::new(e.width, e.height));
        }
    }
}
