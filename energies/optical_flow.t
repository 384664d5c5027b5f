-- Dense optical flow between two grey images: the flow u(i, j) carries pixel (i, j) of
-- the source onto the bilinearly sampled target (whose derivative images give the
-- Jacobian of the sample), plus a 4-neighbour smoothness prior on u. Declaration
-- indices follow the reference example (examples/optical_flow).
local cols, rows = Dim("W", 0), Dim("H", 1)
local fitW = Param("w_fit", float, 0)
local smoothW = Param("w_reg", float, 1)
local flow = Unknown("X", opt_float2, {cols, rows}, 2)
local source = Array("I", opt_float, {cols, rows}, 3)
local tgt = Array("I_hat", opt_float, {cols, rows}, 4)
local tgtDx = Array("I_hat_dx", opt_float, {cols, rows}, 5)
local tgtDy = Array("I_hat_dy", opt_float, {cols, rows}, 6)
local warpedTarget = SampledImage(tgt, tgtDx, tgtDy)

local px, py = Index(0), Index(1)
UsePreconditioner(false)

local brightness = source(0, 0) - warpedTarget(px + flow(0, 0, 0), py + flow(0, 0, 1))
Energy(fitW * brightness)

for sx, sy in Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} } do
    local d = smoothW * (flow(0, 0) - flow(sx, sy))
    Energy(Select(InBounds(sx, sy), d, 0))
end
