-- Poisson image editing: blend the gradients of T into X inside the mask
-- (same energy as the reference's examples/poisson_image_editing/poisson_image_editing.t).
local W, H = Dim("W", 0), Dim("H", 1)
local X = Unknown("X", opt_float4, {W, H}, 0)   -- result, starts as the base image
local T = Array("T", opt_float4, {W, H}, 1)     -- image whose gradients are inserted
local M = Array("M", opt_float, {W, H}, 2)      -- 0 = solve here, otherwise fixed
UsePreconditioner(false)
Exclude(Not(eq(M(0, 0), 0)))

for x, y in Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} } do
    local grad_diff = (X(0, 0) - X(x, y)) - (T(0, 0) - T(x, y))
    Energy(Select(InBounds(x, y), grad_diff, 0))
end
