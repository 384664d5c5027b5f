-- Volumetric denoising on a 3-D grid: stay close to the noisy data, penalise
-- differences between the 6 face neighbours, skip voxels outside the mask.
-- No hand-written kernel family matches this energy: it runs on the kernels the
-- general front end generates (opt_amd/csrc/gen, generic.hip).
local W, H, D = Dim("W", 0), Dim("H", 1), Dim("D", 2)

local X     = Unknown("X", opt_float, {W, H, D}, 0)     -- denoised volume
local Data  = Array("Data", opt_float, {W, H, D}, 1)    -- noisy observation
local Mask  = Array("Mask", opt_float, {W, H, D}, 2)    -- 0 = solve for this voxel
local w_fit = Param("w_fit", float, 3)
local w_reg = Param("w_reg", float, 4)

Exclude(Not(eq(Mask(0, 0, 0), 0)))

Energy(w_fit * (X(0, 0, 0) - Data(0, 0, 0)))
for dx, dy, dz in Stencil { {1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1} } do
    Energy(Select(InBounds(dx, dy, dz), w_reg * (X(0, 0, 0) - X(dx, dy, dz)), 0))
end
