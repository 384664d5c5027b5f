-- As-rigid-as-possible deformation of a regular 3-D lattice (same energy as the
-- reference's examples/volumetric_mesh_deformation; same declaration indices): every
-- lattice edge keeps its rest vector up to the rotation of its first end.
local W, H, D = Dim("W", 0), Dim("H", 1), Dim("D", 2)

local Offset      = Unknown("Offset", opt_float3, {W, H, D}, 0)
local Angle       = Unknown("Angle", opt_float3, {W, H, D}, 1)
local UrShape     = Array("UrShape", opt_float3, {W, H, D}, 2)
local Constraints = Array("Constraints", opt_float3, {W, H, D}, 3)
local w_fit = Param("w_fitSqrt", float, 4)
local w_reg = Param("w_regSqrt", float, 5)
UsePreconditioner(true)

local has_target = greatereq(Constraints(0, 0, 0)(0), -999999.9)
Energy(Select(has_target, w_fit * (Offset(0, 0, 0) - Constraints(0, 0, 0)), 0))

for dx, dy, dz in Stencil { {1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1} } do
    local edge = (Offset(0, 0, 0) - Offset(dx, dy, dz))
               - Rotate3D(Angle(0, 0, 0), UrShape(0, 0, 0) - UrShape(dx, dy, dz))
    Energy(w_reg * Select(InBounds(0, 0, 0), Select(InBounds(dx, dy, dz), edge, 0.0), 0.0))
end
