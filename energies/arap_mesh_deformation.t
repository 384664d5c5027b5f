-- As-rigid-as-possible deformation of a triangle mesh given as a vertex graph.
-- Unknowns: the deformed position and an Euler-angle rotation per vertex. Handles pull
-- their vertex towards a target; every directed edge (a -> b) should keep its rest
-- vector up to the rotation of a. Declaration indices follow the reference example
-- (examples/arap_mesh_deformation), so its problemparams bind unchanged.
local vertexCount, edgeCount = Dim("N", 0), Dim("NUMEDGES", 1)

local fitWeight = Param("w_fitSqrt", float, 0)
local rigidWeight = Param("w_regSqrt", float, 1)
local pos = Unknown("Offset", opt_float3, {vertexCount}, 2)
local euler = Unknown("Angle", opt_float3, {vertexCount}, 3)
local rest = Array("UrShape", opt_float3, {vertexCount}, 4)
local target = Array("Constraints", opt_float3, {vertexCount}, 5)   -- x < -999999.9: free
local edges = Graph("G", {edgeCount}, "v0", {vertexCount}, 7, "v1", {vertexCount}, 8)
UsePreconditioner(true)

local function handle_term()
    local pull = pos(0) - target(0)
    local pinned = greatereq(target(0, 0), -999999.9)   -- (0, 0) on a 1-D array: channel 0
    return Select(pinned, fitWeight * pull, 0)
end

local function rigidity_term(a, b)
    local moved = pos(a) - pos(b)
    local rotated = Rotate3D(euler(a), rest(a) - rest(b))
    return rigidWeight * (moved - rotated)
end

Energy(handle_term())
Energy(rigidity_term(edges.v0, edges.v1))
