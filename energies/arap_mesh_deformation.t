-- As-rigid-as-possible mesh deformation on a vertex graph (same energy as the
-- reference's examples/arap_mesh_deformation/arap_mesh_deformation.t, same indices).
local N = Dim("N", 0)
local NUMEDGES = Dim("NUMEDGES", 1)

local w_fitSqrt = Param("w_fitSqrt", float, 0)
local w_regSqrt = Param("w_regSqrt", float, 1)
local Offset = Unknown("Offset", opt_float3, {N}, 2)        -- deformed vertex positions
local Angle = Unknown("Angle", opt_float3, {N}, 3)          -- per-vertex rotation (Euler)
local UrShape = Array("UrShape", opt_float3, {N}, 4)        -- rest positions
local Constraints = Array("Constraints", opt_float3, {N}, 5) -- targets (-inf: free)
local G = Graph("G", {NUMEDGES}, "v0", {N}, 7, "v1", {N}, 8)
UsePreconditioner(true)

-- handles pull their vertex to the target
local has_target = greatereq(Constraints(0, 0), -999999.9)
Energy(Select(has_target, w_fitSqrt * (Offset(0) - Constraints(0)), 0))

-- every edge keeps its rest shape up to the rotation of its first vertex
local rigid = (Offset(G.v0) - Offset(G.v1)) - Rotate3D(Angle(G.v0), UrShape(G.v0) - UrShape(G.v1))
Energy(w_regSqrt * rigid)
